// gpushare-comgr-warm: the first-stream work of a HIP process, against the system HIP runtime,
// run once by the DaemonSet's init container with AMD_COMGR_CACHE set
// (aliyun_gpushare_device_plugin_amd/quota/comgr_cache.py). The runtime builds its blit (copy and
// fill) kernels with comgr at a process's first stream; comgr's cache keeps what it built, so a
// container whose runtime is the same finds them there instead of compiling them (~110 ms of its
// start-up, profiles/r5/comgr_cache/). Prints one JSON line: what ran and how long it took.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                                        \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) {                                                                          \
      std::printf("{\"ok\": false, \"step\": \"%s\", \"error\": \"%s\"}\n", #x, hipGetErrorString(e_)); \
      return 1;                                                                                      \
    }                                                                                                \
  } while (0)

int main(int argc, char** argv) {
  int dev = argc > 1 ? std::atoi(argv[1]) : 0;
  double t0 = now_ms();
  int rtv = 0;
  CK(hipRuntimeGetVersion(&rtv));
  CK(hipSetDevice(dev));
  double t1 = now_ms();
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const size_t n = 4 << 20;
  void *d0 = nullptr, *d1 = nullptr, *h = nullptr;
  CK(hipMalloc(&d0, n));
  CK(hipMalloc(&d1, n));
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  // every blit the runtime offers: fills of each width, linear and 2-D copies in each direction
  CK(hipMemsetAsync(d0, 0, n, s));
  CK(hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(d0), 1, n / 2, s));
  CK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d0), 2, n / 4, s));
  CK(hipMemcpyAsync(d1, d0, n, hipMemcpyDeviceToDevice, s));
  CK(hipMemcpyAsync(h, d0, n, hipMemcpyDeviceToHost, s));
  CK(hipMemcpyAsync(d0, h, n, hipMemcpyHostToDevice, s));
  CK(hipMemcpy2DAsync(d1, 1024, d0, 1024, 512, 64, hipMemcpyDeviceToDevice, s));
  CK(hipMemset2DAsync(d1, 1024, 3, 512, 64, s));
  CK(hipStreamSynchronize(s));
  CK(hipMemset(d0, 0, n));  // the null stream
  CK(hipDeviceSynchronize());
  double t2 = now_ms();
  CK(hipHostFree(h));
  CK(hipFree(d1));
  CK(hipFree(d0));
  CK(hipStreamDestroy(s));
  std::printf("{\"ok\": true, \"runtime\": \"system\", \"runtime_version\": %d, \"init_ms\": %.3f, \"first_stream_ms\": %.3f}\n",
              rtv, t1 - t0, t2 - t1);
  return 0;
}
