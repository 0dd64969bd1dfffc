// The HBM broker's scrub: zero granules at HBM write bandwidth.
//
// Built as a code object (hipcc --genco --offload-arch=gfx950) next to the broker, which loads it
// with hipModuleLoad and launches it on its own stream. The broker is host code built by g++; it
// falls back to hipMemsetAsync when the code object is missing.
//
// Pure streaming stores: each lane writes 16 B per iteration (global_store_dwordx4), non-temporal,
// so the zeroes do not displace tenants' data in L2 / MALL. A grid-stride loop over 64-wide
// waves, 256 threads per block, grid sized by the caller to fill the 256 CUs several times over.
// Nothing is read. Stores go through the vector memory path only.
#include <hip/hip_runtime.h>

#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

extern "C" __global__ void __launch_bounds__(256) gs_scrub(u32x4* __restrict__ p, uint64_t n16) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  uint64_t i = uint64_t(blockIdx.x) * 256u + threadIdx.x;
  const uint64_t stride = uint64_t(gridDim.x) * 256u;
  // 4 stores in flight per lane per iteration
  for (; i + 3 * stride < n16; i += 4 * stride) {
    __builtin_nontemporal_store(z, p + i);
    __builtin_nontemporal_store(z, p + i + stride);
    __builtin_nontemporal_store(z, p + i + 2 * stride);
    __builtin_nontemporal_store(z, p + i + 3 * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(z, p + i);
}

// Up to 8 ranges in one dispatch: each granule has an address range of its own (so the driver
// gets its memory back when the broker frees it), so a chunk of released granules is rarely one
// contiguous range, and a dispatch per granule pays the grid's ramp-up and drain every GiB
// (4.4 TB/s per 1 GiB dispatch against 6.7 TB/s for 8 GiB, profiles/r6/scrub_kernel.md). Block b
// zeroes range b % count; the caller makes the grid a multiple of count.
struct ScrubSet {
  u32x4* p[8];
  uint64_t n16[8];
  uint32_t count;
};

extern "C" __global__ void __launch_bounds__(256) gs_scrub_n(ScrubSet s) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  const uint32_t r = blockIdx.x % s.count;
  u32x4* __restrict__ p = s.p[r];
  const uint64_t n16 = s.n16[r];
  uint64_t i = uint64_t(blockIdx.x / s.count) * 256u + threadIdx.x;
  const uint64_t stride = uint64_t(gridDim.x / s.count) * 256u;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    __builtin_nontemporal_store(z, p + i);
    __builtin_nontemporal_store(z, p + i + stride);
    __builtin_nontemporal_store(z, p + i + 2 * stride);
    __builtin_nontemporal_store(z, p + i + 3 * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(z, p + i);
}
