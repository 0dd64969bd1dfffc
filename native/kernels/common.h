// Shared helpers for the gfx950 (CDNA4) kernels of libgpushare_kernels.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4_t __attribute__((ext_vector_type(4)));

#define GS_KERNEL_API extern "C" __attribute__((visibility("default")))

// bf16 <-> f32 (bit-level, round-to-nearest-even; NaN handled by the compiler's cvt where it
// matters — MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
  return __uint_as_float(((unsigned)h) << 16);
}
__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;  // lowers to v_cvt_pk_bf16_f32 on gfx950 (NaN-preserving)
  return __builtin_bit_cast(unsigned short, b);
}

__device__ __forceinline__ float silu_f32(float x) { return x / (1.0f + __expf(-x)); }

// Wave-wide sum (64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Error codes returned by the C launchers.
enum { GS_OK = 0, GS_EINVAL = 1, GS_ELAUNCH = 2 };

inline int gs_launch_status() { return hipGetLastError() == hipSuccess ? GS_OK : GS_ELAUNCH; }

// 4-wave GEMM launcher (gemm_bf16_w4.hip); GS_EINVAL when the shape or output layout does not
// suit it (M % 256, N % 256, K % 128, ldc % 8, 16-B aligned C).
int gs_gemm_w4_launch(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                      int lda, int ldb, int ldc, int flags, hipStream_t stream, int reps = 1);
