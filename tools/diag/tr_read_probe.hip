// Diagnostic: measure ds_read_b64_tr_b16 lane semantics on gfx950.
// LDS holds a 16x64 u16 matrix M[r][c] = r*256 + c. Lane l supplies the address of
// row R(l), columns C(l)..C(l)+3 (pattern A: R = (l&15)>>2 + 4*(l>>4), C = 4*(l&3)).
// Prints, for each lane, the 4 returned values decoded as (row, col).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void probe(int* out) {
  __shared__ unsigned short M[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) M[i] = (unsigned short)((i / 64) * 256 + (i % 64));
  __syncthreads();
  int l = threadIdx.x;
  int R = ((l & 15) >> 2) + 4 * (l >> 4), C = 4 * (l & 3);
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(M + R * 64 + C));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = (unsigned short)v[e];
}
int main() {
  int* d; hipMalloc(&d, 64 * 4 * sizeof(int));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  int h[256]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int e = 0; e < 4; ++e) printf(" (r%d,c%d)", h[l * 4 + e] / 256, h[l * 4 + e] % 256);
    printf("\n");
  }
  return 0;
}
