// Diagnostic: v_mfma_f32_16x16x32_bf16 with operands built three ways, vs host reference.
//  mode 0: A and B loaded from memory as bf16x8 (lane l: row l&15, k = 8*(l>>4) + j)
//  mode 1: B built element-wise from floats via (__bf16) casts
//  mode 2: A built element-wise via bit_cast of shorts (like a transposed-read result)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include <string.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const unsigned short* A, const unsigned short* B, const float* Bf, float* D, int mode) {
  int l = threadIdx.x, r = l & 15, g = l >> 4;
  bf16x8 a = *(const bf16x8*)(A + r * 32 + 8 * g);       // A[16][32]
  bf16x8 b = *(const bf16x8*)(B + r * 32 + 8 * g);       // B^T stored [16 cols][32 k]
  if (mode == 1) {
    for (int j = 0; j < 8; ++j) b[j] = (__bf16)Bf[r * 32 + 8 * g + j];
  } else if (mode == 2) {
    for (int j = 0; j < 8; ++j) { short s = (short)A[r * 32 + 8 * g + j]; a[j] = __builtin_bit_cast(__bf16, s); }
  }
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[(4 * g + i) * 16 + r] = acc[i];   // D[row][col]
}
static unsigned short f2b(float f) { unsigned u; memcpy(&u, &f, 4); return (unsigned short)(u >> 16); }
static float b2f(unsigned short h) { unsigned u = (unsigned)h << 16; float f; memcpy(&f, &u, 4); return f; }
int main() {
  unsigned short hA[512], hB[512]; float hBf[512], ref[256];
  for (int i = 0; i < 512; ++i) { hA[i] = f2b((float)((i * 7) % 13 - 6)); hBf[i] = (float)((i * 5) % 11 - 5); hB[i] = f2b(hBf[i]); }
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { float s = 0; for (int k = 0; k < 32; ++k) s += b2f(hA[i * 32 + k]) * b2f(hB[j * 32 + k]); ref[i * 16 + j] = s; }
  unsigned short *dA, *dB; float *dBf, *dD;
  (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dBf, 2048); (void)hipMalloc(&dD, 1024);
  (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  (void)hipMemcpy(dBf, hBf, 2048, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dBf, dD, mode);
    float hD[256]; (void)hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
    float err = 0; for (int i = 0; i < 256; ++i) err = fmaxf(err, fabsf(hD[i] - ref[i]));
    printf("mode %d max err %g  D[0][0..3]=%g %g %g %g ref=%g %g %g %g\n", mode, err, hD[0], hD[1], hD[2], hD[3], ref[0], ref[1], ref[2], ref[3]);
  }
  return 0;
}
