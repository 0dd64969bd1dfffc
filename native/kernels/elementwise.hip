// Memory-bound fused kernels for the demo Llama workload (bf16, 16-byte vector I/O).
//  * gs_rmsnorm_bf16:  [h = x + r  (written to r_out)]  y = h * rsqrt(mean(h^2) + eps) * w
//  * gs_silu_mul_bf16: y[m, f] = silu(gu[m, f]) * gu[m, F + f]   (gate|up concatenated;
//                      gs_silu_mul_il_bf16: the interleaved-by-16 layout)
//  * gs_rope_bf16:     in-place rotate-half RoPE on q/k with host-precomputed cos/sin tables
//  * gs_argmax_rows_bf16: greedy sampling, out[b] = argmax_v x[b, v] as torch.argmax defines it
//                      (first index of the maximum; NaN counts as the maximum)
// Per cdna_hip_programming.md Appendix B: vectorised 16-B loads, f32 math, trig from a
// table (no on-device sin/cos), one row per 256-thread block for the row reductions.
#include "common.h"

namespace {

constexpr int RMS_THREADS = 256;

__global__ __launch_bounds__(RMS_THREADS) void rmsnorm_bf16(const unsigned short* __restrict__ x,
                                                            const unsigned short* __restrict__ resid_in,
                                                            unsigned short* __restrict__ resid_out,
                                                            const unsigned short* __restrict__ w,
                                                            unsigned short* __restrict__ y, int H, float eps) {
  const int row = blockIdx.x;
  const size_t base = (size_t)row * H;
  const int nvec = H / 8;
  // H <= 8 * 256 * 4 = 8192 values per row held in registers (4 vectors per thread)
  constexpr int MAXV = 4;
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int t = 0; t < MAXV; ++t) {
    const int vi = threadIdx.x + t * RMS_THREADS;
    if (vi < nvec) {
      const u16x8_t xv = *(const u16x8_t*)(x + base + vi * 8);
      if (resid_in) {
        const u16x8_t rv = *(const u16x8_t*)(resid_in + base + vi * 8);
        u16x8_t hv;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float h = bf16_to_f32(xv[e]) + bf16_to_f32(rv[e]);
          hv[e] = f32_to_bf16(h);
          v[t][e] = bf16_to_f32(hv[e]);  // normalise exactly what is stored as the residual
        }
        *(u16x8_t*)(resid_out + base + vi * 8) = hv;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[t][e] = bf16_to_f32(xv[e]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[t][e] * v[t][e];
    }
  }
  __shared__ float red[RMS_THREADS / 64];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int i = 0; i < RMS_THREADS / 64; ++i) tot += red[i];
  const float inv = rsqrtf(tot / (float)H + eps);
#pragma unroll
  for (int t = 0; t < MAXV; ++t) {
    const int vi = threadIdx.x + t * RMS_THREADS;
    if (vi < nvec) {
      const u16x8_t wv = *(const u16x8_t*)(w + vi * 8);
      u16x8_t o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(v[t][e] * inv * bf16_to_f32(wv[e]));
      *(u16x8_t*)(y + base + vi * 8) = o;
    }
  }
}

__global__ __launch_bounds__(256) void silu_mul_bf16(const unsigned short* __restrict__ gu,
                                                     unsigned short* __restrict__ y, int M, int F, int il) {
  const int nvec = F / 8;
  const size_t total = (size_t)M * nvec;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i / nvec, f = (i % nvec) * 8;
    // il: gate/up rows interleaved by 16 (ops.interleave_gate_up): feature f's gate sits at
    // column (f / 16) * 32 + f % 16 and its up 16 columns later
    const size_t go = il ? (f / 16) * 32 + f % 16 : f, uo = il ? go + 16 : F + f;
    const u16x8_t g = *(const u16x8_t*)(gu + m * 2 * F + go);
    const u16x8_t u = *(const u16x8_t*)(gu + m * 2 * F + uo);
    u16x8_t o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(silu_f32(bf16_to_f32(g[e])) * bf16_to_f32(u[e]));
    *(u16x8_t*)(y + m * F + f) = o;
  }
}

// x: [T, nheads, D] with row stride `stride` (elements) between tokens; pos[t] or t % S.
__global__ __launch_bounds__(256) void rope_bf16(unsigned short* __restrict__ x, const float* __restrict__ cosb,
                                                 const float* __restrict__ sinb, const int* __restrict__ pos,
                                                 int T, int nheads, int D, int stride, int S) {
  const int half = D / 2, nq = half / 4;  // 4 pairs per thread
  const size_t total = (size_t)T * nheads * nq;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int qd = (int)(i % nq);
    const size_t th = i / nq;
    const int h = (int)(th % nheads);
    const int t = (int)(th / nheads);
    const int p = pos ? pos[t] : (t % S);
    unsigned short* row = x + (size_t)t * stride + (size_t)h * D;
    const int d = qd * 4;
    const u16x4_t a = *(const u16x4_t*)(row + d);
    const u16x4_t b = *(const u16x4_t*)(row + half + d);
    const float4 c = *(const float4*)(cosb + (size_t)p * half + d);
    const float4 s = *(const float4*)(sinb + (size_t)p * half + d);
    const float cc[4] = {c.x, c.y, c.z, c.w}, sc[4] = {s.x, s.y, s.z, s.w};
    u16x4_t oa, ob;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x1 = bf16_to_f32(a[e]), x2 = bf16_to_f32(b[e]);
      oa[e] = f32_to_bf16(x1 * cc[e] - x2 * sc[e]);
      ob[e] = f32_to_bf16(x2 * cc[e] + x1 * sc[e]);
    }
    *(u16x4_t*)(row + d) = oa;
    *(u16x4_t*)(row + half + d) = ob;
  }
}

inline int grid_for(size_t work, int threads) {
  size_t b = (work + threads - 1) / threads;
  return (int)(b < 2048 * 8 ? (b ? b : 1) : 2048 * 8);
}

// Order-preserving 32-bit key of a bf16 value (NaN above +inf); with the index complemented in the
// low half, the max of (key << 32 | ~idx) is the first index of the maximum.
__device__ __forceinline__ unsigned long long argmax_key(unsigned short h, int idx) {
  unsigned u = ((unsigned)h) << 16;
  const bool nan = (u & 0x7fffffffu) > 0x7f800000u;
  u = nan ? 0xffffffffu : (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned)~idx;
}

// One 1024-thread workgroup per row: the decode step's logits row (128256 entries for Llama 3) is
// read with 16-B loads, 4 in flight per thread, and reduced in registers, then across the waves.
constexpr int AM_THREADS = 1024;
__global__ __launch_bounds__(AM_THREADS) void argmax_rows_bf16(const unsigned short* __restrict__ x, int ld, int V,
                                                               long long* __restrict__ out) {
  const unsigned short* r = x + (size_t)blockIdx.x * ld;
  const int tid = threadIdx.x, v8 = V / 8;
  unsigned long long best = 0;
  int v = tid;
  for (; v + 3 * AM_THREADS < v8; v += 4 * AM_THREADS) {
    u16x8_t q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = *(const u16x8_t*)(r + (size_t)(v + j * AM_THREADS) * 8);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const unsigned long long k = argmax_key(q[j][e], (v + j * AM_THREADS) * 8 + e);
        best = k > best ? k : best;
      }
  }
  for (; v < v8; v += AM_THREADS) {
    const u16x8_t q = *(const u16x8_t*)(r + (size_t)v * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const unsigned long long k = argmax_key(q[e], v * 8 + e);
      best = k > best ? k : best;
    }
  }
  for (int t = v8 * 8 + tid; t < V; t += AM_THREADS) {
    const unsigned long long k = argmax_key(r[t], t);
    best = k > best ? k : best;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long k = __shfl_xor(best, o, 64);
    best = k > best ? k : best;
  }
  __shared__ unsigned long long red[AM_THREADS / 64];
  if ((tid & 63) == 0) red[tid >> 6] = best;
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int w = 1; w < AM_THREADS / 64; ++w) best = red[w] > best ? red[w] : best;
    out[blockIdx.x] = (long long)(unsigned)~(unsigned)(best & 0xffffffffu);
  }
}

}  // namespace

GS_KERNEL_API int gs_argmax_rows_bf16(const void* x, int ld, int B, int V, void* out, hipStream_t stream) {
  if (B <= 0 || V <= 0 || ld < V || ld % 8 || ((uintptr_t)x & 15)) return GS_EINVAL;
  hipLaunchKernelGGL(argmax_rows_bf16, dim3(B), dim3(AM_THREADS), 0, stream, (const unsigned short*)x, ld, V,
                     (long long*)out);
  return gs_launch_status();
}

GS_KERNEL_API int gs_rmsnorm_bf16(const void* x, const void* resid_in, void* resid_out, const void* w, void* y,
                                  int M, int H, float eps, hipStream_t stream) {
  if (M <= 0 || H <= 0 || H % 8 || H > 8 * RMS_THREADS * 4 || (resid_in && !resid_out)) return GS_EINVAL;
  hipLaunchKernelGGL(rmsnorm_bf16, dim3(M), dim3(RMS_THREADS), 0, stream, (const unsigned short*)x,
                     (const unsigned short*)resid_in, (unsigned short*)resid_out, (const unsigned short*)w,
                     (unsigned short*)y, H, eps);
  return gs_launch_status();
}

GS_KERNEL_API int gs_silu_mul_bf16(const void* gu, void* y, int M, int F, hipStream_t stream) {
  if (M <= 0 || F <= 0 || F % 8) return GS_EINVAL;
  hipLaunchKernelGGL(silu_mul_bf16, dim3(grid_for((size_t)M * F / 8, 256)), dim3(256), 0, stream,
                     (const unsigned short*)gu, (unsigned short*)y, M, F, 0);
  return gs_launch_status();
}

// Same on the interleaved-by-16 gate/up layout the SwiGLU weights use (no de-interleave copy).
GS_KERNEL_API int gs_silu_mul_il_bf16(const void* gu, void* y, int M, int F, hipStream_t stream) {
  if (M <= 0 || F <= 0 || F % 16) return GS_EINVAL;
  hipLaunchKernelGGL(silu_mul_bf16, dim3(grid_for((size_t)M * F / 8, 256)), dim3(256), 0, stream,
                     (const unsigned short*)gu, (unsigned short*)y, M, F, 1);
  return gs_launch_status();
}

GS_KERNEL_API int gs_rope_bf16(void* x, const float* cosb, const float* sinb, const int* pos, int T, int nheads,
                               int D, int stride, int S, hipStream_t stream) {
  if (T <= 0 || nheads <= 0 || D % 8 || stride < nheads * D || S <= 0) return GS_EINVAL;
  hipLaunchKernelGGL(rope_bf16, dim3(grid_for((size_t)T * nheads * (D / 8), 256)), dim3(256), 0, stream,
                     (unsigned short*)x, cosb, sinb, pos, T, nheads, D, stride, S);
  return gs_launch_status();
}
