// Does HBM a process created with hipMemCreate (and exported as a dma-buf) go back to the driver
// when the process unmaps, releases and closes it — without exiting? The broker's SIZE 0 path
// (native/hbmbroker/hbmbroker.cpp destroy_granule) depends on it. Prints one JSON line per
// variant: device free before, after creating N granules, after destroying them (at once and
// after 2 s).
//
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/release_probe tools/diag/release_probe.cpp
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

static size_t dev_free() {
  size_t f = 0, t = 0;
  CK(hipMemGetInfo(&f, &t));
  return f;
}

int main(int argc, char** argv) {
  int n = argc > 1 ? std::atoi(argv[1]) : 8;
  const char* variant = argc > 2 ? argv[2] : "broker";
  bool do_export = std::strcmp(variant, "noexport") != 0;
  bool do_map = std::strcmp(variant, "nomap") != 0;
  bool close_first = std::strcmp(variant, "close_first") == 0;
  bool touch = std::strcmp(variant, "touch") == 0 || std::strcmp(variant, "broker") == 0;
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  bool pergran = std::strcmp(variant, "pergran") == 0;
  const size_t gran = 1ull << 30;
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t f0 = dev_free();
  if (pergran) {  // a range of its own per granule: give half back, range and all
    std::vector<char*> va(n);
    std::vector<hipMemGenericAllocationHandle_t> hh(n);
    std::vector<int> ff(n, -1);
    hipMemAccessDesc d{};
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = 0;
    d.flags = hipMemAccessFlagsProtReadWrite;
    for (int i = 0; i < n; ++i) {
      CK(hipMemCreate(&hh[i], gran, &prop, 0));
      CK(hipMemExportToShareableHandle(&ff[i], hh[i], hipMemHandleTypePosixFileDescriptor, 0));
      CK(hipMemAddressReserve(reinterpret_cast<void**>(&va[i]), gran, 0, nullptr, 0));
      CK(hipMemMap(va[i], gran, 0, hh[i], 0));
      CK(hipMemSetAccess(va[i], gran, &d, 1));
      CK(hipMemsetD8(reinterpret_cast<hipDeviceptr_t>(va[i]), 0, gran));
    }
    CK(hipDeviceSynchronize());
    size_t g1 = dev_free();
    for (int i = 0; i < n / 2; ++i) {
      CK(hipMemUnmap(va[i], gran));
      CK(hipMemRelease(hh[i]));
      CK(hipMemAddressFree(va[i], gran));
      close(ff[i]);
    }
    size_t g2 = dev_free();
    std::printf("{\"variant\": \"pergran\", \"n\": %d, \"free_gib\": [%.2f, %.2f, %.2f]}\n", n, f0 / 1073741824.0,
                g1 / 1073741824.0, g2 / 1073741824.0);
    return 0;
  }
  char* base = nullptr;
  CK(hipMemAddressReserve(reinterpret_cast<void**>(&base), gran * n, 0, nullptr, 0));
  std::vector<hipMemGenericAllocationHandle_t> h(n);
  std::vector<int> fd(n, -1);
  for (int i = 0; i < n; ++i) {
    CK(hipMemCreate(&h[i], gran, &prop, 0));
    if (do_export) CK(hipMemExportToShareableHandle(&fd[i], h[i], hipMemHandleTypePosixFileDescriptor, 0));
    if (do_map) CK(hipMemMap(base + size_t(i) * gran, gran, 0, h[i], 0));
  }
  if (do_map) {
    hipMemAccessDesc d{};
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = 0;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(base, gran * n, &d, 1));
    if (touch) {
      CK(hipMemsetD8(reinterpret_cast<hipDeviceptr_t>(base), 0, gran * n));
      CK(hipDeviceSynchronize());
    }
  }
  size_t f1 = dev_free();
  for (int i = 0; i < n; ++i) {
    if (close_first && fd[i] >= 0) close(fd[i]), fd[i] = -1;
    if (do_map) CK(hipMemUnmap(base + size_t(i) * gran, gran));
    CK(hipMemRelease(h[i]));
    if (fd[i] >= 0) close(fd[i]), fd[i] = -1;
  }
  size_t f2 = dev_free();
  sleep(2);
  size_t f3 = dev_free();
  CK(hipMemAddressFree(base, gran * n));
  size_t f4 = dev_free();
  std::printf("{\"variant\": \"%s\", \"n\": %d, \"free_gib\": [%.2f, %.2f, %.2f, %.2f, %.2f]}\n", variant, n,
              f0 / 1073741824.0, f1 / 1073741824.0, f2 / 1073741824.0, f3 / 1073741824.0, f4 / 1073741824.0);
  return 0;
}
