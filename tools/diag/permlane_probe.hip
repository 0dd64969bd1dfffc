// Probe: semantics of __builtin_amdgcn_permlane32_swap (v_permlane32_swap_b32) on gfx950.
// Lane i passes a = i, b = 100 + i; prints what each lane gets back in r[0] and r[1].
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* o) {
  unsigned i = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(i, 100u + i, false, false);
  o[2 * i] = r[0];
  o[2 * i + 1] = r[1];
}
int main() {
  unsigned* d;
  unsigned h[128];
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  k<<<1, 64>>>(d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int i : {0, 1, 31, 32, 33, 63}) printf("lane %d: r0=%u r1=%u\n", i, h[2 * i], h[2 * i + 1]);
  hipFree(d);
  return 0;
}
