// CU census: where do a launch's workgroups run? Used to verify compute isolation on hardware
// (alloc/cuslots.py): every workgroup records its XCD (HW_REG_XCC_ID) and its shader-engine /
// CU coordinates (HW_REG_HW_ID), after a short s_sleep so the grid spreads over every CU the
// queue's CU mask allows instead of being absorbed by the first CUs to come free.
#include "common.h"

namespace {

// s_getreg immediates: register id | offset << 6 | (size - 1) << 11
constexpr int kHwIdReg = 4 | (0 << 6) | (31 << 11);   // HW_REG_HW_ID
constexpr int kXccIdReg = 20 | (0 << 6) | (15 << 11); // HW_REG_XCC_ID (gfx942 / gfx950)

__global__ __launch_bounds__(64) void cu_census(unsigned* __restrict__ out, int spin) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg(kHwIdReg);
    const unsigned xcc = __builtin_amdgcn_s_getreg(kXccIdReg) & 0xf;
    out[blockIdx.x] = (xcc << 16) | (hw & 0xffff);   // SE [15:13], SH [12], CU [11:8]
  }
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(127);
}

}  // namespace

// out[nblocks]: (xcc << 16) | HW_ID[15:0] per workgroup. spin: s_sleep(127) repeats per block.
GS_KERNEL_API int gs_cu_census(void* out, int nblocks, int spin, hipStream_t stream) {
  if (!out || nblocks <= 0 || nblocks > (1 << 20) || spin < 0 || spin > 64) return GS_EINVAL;
  hipLaunchKernelGGL(cu_census, dim3(nblocks), dim3(64), 0, stream, (unsigned*)out, spin);
  return gs_launch_status();
}
