// Quota-shim probe for a real MI355X: run under LD_PRELOAD=libgpushare_hipquota.so (and,
// optionally, rocprofv3 --memory-allocation-trace). Each command prints one JSON line with the
// shim ledger's view ("used", from gpushare_shim_stats) next to the device's own view (the
// runtime's real hipMemGetInfo, looked up in libamdhip64 itself so the shim's quota-limited
// report does not hide it). Commands:
//   granule             hipMalloc of sizes around the 2 MiB fragment: charge vs HBM consumed
//   pool BYTES          stream-ordered pool (release threshold = max): alloc, free, sync, trim
//   array BYTES         hipMallocArray of ~BYTES (float4 texels), then hipFreeArray
//   scratch KB          a kernel whose lanes each use KB KiB of private (scratch) memory
//   alloc BYTES         plain hipMalloc (keeps it), prints rc
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef int (*stats_fn)(uint64_t*, uint64_t*, uint64_t*, uint64_t*);
typedef hipError_t (*meminfo_fn)(size_t*, size_t*);

static stats_fn g_stats;
static meminfo_fn g_real_info;

static uint64_t used() {
  uint64_t u = 0, q = 0, d = 0, p = 0;
  if (g_stats) g_stats(&u, &q, &d, &p);
  return u;
}
static uint64_t denied() {
  uint64_t u = 0, q = 0, d = 0, p = 0;
  if (g_stats) g_stats(&u, &q, &d, &p);
  return d;
}
static size_t dev_used() {
  size_t f = 0, t = 0;
  if (g_real_info) g_real_info(&f, &t);
  return t - f;
}

// Dynamic indexing into a per-lane array forces it into scratch (private segment) memory.
template <int N>
__global__ void scratch_kernel(float* out, int salt) {
  float buf[N];
  int t = threadIdx.x + blockIdx.x * blockDim.x;
  for (int i = 0; i < N; ++i) buf[i] = (float)(i ^ salt ^ t);
  float acc = 0.f;
  for (int i = 0; i < N; i += 61) acc += buf[(i * 37 + t) % N];
  out[t] = acc;
}

int main(int argc, char** argv) {
  g_stats = (stats_fn)dlsym(RTLD_DEFAULT, "gpushare_shim_stats");
  void* hip = dlopen("libamdhip64.so.7", RTLD_NOLOAD | RTLD_LAZY);
  if (!hip) hip = dlopen("libamdhip64.so", RTLD_NOLOAD | RTLD_LAZY);
  g_real_info = hip ? (meminfo_fn)dlsym(hip, "hipMemGetInfo") : nullptr;
  if (hipSetDevice(0) != hipSuccess) return 2;
  void* warm = nullptr;
  (void)hipMalloc(&warm, 1);   // runtime pools and first fragment exist before measuring
  (void)hipFree(warm);
  (void)hipDeviceSynchronize();
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "granule")) {
      size_t sizes[] = {1, 4096, 65536, (2u << 20) - 1, 2u << 20, (2u << 20) + 1, 3u << 20, (6u << 20) + 4096,
                        64u << 20};
      for (size_t s : sizes) {
        uint64_t u0 = used();
        size_t d0 = dev_used();
        void* p = nullptr;
        int rc = hipMalloc(&p, s);
        uint64_t u1 = used();
        size_t d1 = dev_used();
        printf("{\"op\":\"granule\",\"requested\":%zu,\"rc\":%d,\"shim_charge\":%llu,\"device_bytes\":%lld}\n", s, rc,
               (unsigned long long)(u1 - u0), (long long)(d1 - d0));
        fflush(stdout);
        (void)hipFree(p);
      }
    } else if (!strcmp(argv[i], "pool")) {
      size_t n = strtoull(argv[++i], 0, 10);
      hipMemPoolProps props = {};
      props.allocType = hipMemAllocationTypePinned;
      props.location.type = hipMemLocationTypeDevice;
      props.location.id = 0;
      hipMemPool_t pool;
      int rc = hipMemPoolCreate(&pool, &props);
      uint64_t thr = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
      hipStream_t s;
      (void)hipStreamCreate(&s);
      uint64_t u0 = used();
      void* p = nullptr;
      int rc1 = hipMallocFromPoolAsync(&p, n, pool, s);
      (void)hipStreamSynchronize(s);
      uint64_t u1 = used();
      int rc2 = hipFreeAsync(p, s);
      (void)hipStreamSynchronize(s);
      uint64_t u2 = used();
      int rc3 = hipMemPoolTrimTo(pool, 0);
      (void)hipDeviceSynchronize();
      uint64_t u3 = used();
      printf("{\"op\":\"pool\",\"n\":%zu,\"rc\":[%d,%d,%d,%d],\"used_before\":%llu,\"after_alloc\":%llu,"
             "\"after_free\":%llu,\"after_trim\":%llu}\n", n, rc, rc1, rc2, rc3, (unsigned long long)u0,
             (unsigned long long)u1, (unsigned long long)u2, (unsigned long long)u3);
      (void)hipMemPoolDestroy(pool);
      (void)hipStreamDestroy(s);
    } else if (!strcmp(argv[i], "array")) {
      size_t n = strtoull(argv[++i], 0, 10);
      size_t w = 16384, h = n / (w * 16);
      hipChannelFormatDesc desc = hipCreateChannelDesc<float4>();
      hipArray_t arr = nullptr;
      uint64_t u0 = used();
      int rc = hipMallocArray(&arr, &desc, w, h, 0);
      uint64_t u1 = used();
      int rc2 = arr ? hipFreeArray(arr) : -1;
      uint64_t u2 = used();
      printf("{\"op\":\"array\",\"bytes\":%zu,\"rc\":[%d,%d],\"used_before\":%llu,\"after_alloc\":%llu,"
             "\"after_free\":%llu,\"denied\":%llu}\n", w * h * 16, rc, rc2, (unsigned long long)u0,
             (unsigned long long)u1, (unsigned long long)u2, (unsigned long long)denied());
    } else if (!strcmp(argv[i], "scratch")) {
      int kb = atoi(argv[++i]);
      float* out = nullptr;
      int blocks = 256 * 8, threads = 256;
      (void)hipMalloc(&out, sizeof(float) * blocks * threads);
      uint64_t u0 = used();
      size_t d0 = dev_used();
      if (kb >= 16) hipLaunchKernelGGL(scratch_kernel<4096>, dim3(blocks), dim3(threads), 0, 0, out, 7);
      else hipLaunchKernelGGL(scratch_kernel<1024>, dim3(blocks), dim3(threads), 0, 0, out, 7);
      int rc = hipGetLastError();
      int rc2 = hipDeviceSynchronize();
      uint64_t u1 = used();
      size_t d1 = dev_used();
      printf("{\"op\":\"scratch\",\"kb_per_lane\":%d,\"rc\":[%d,%d],\"used_before\":%llu,\"after_launch\":%llu,"
             "\"device_delta\":%lld,\"denied\":%llu}\n", kb >= 16 ? 16 : 4, rc, rc2, (unsigned long long)u0,
             (unsigned long long)u1, (long long)(d1 - d0), (unsigned long long)denied());
      (void)hipFree(out);
    } else if (!strcmp(argv[i], "smalls")) {
      int n = atoi(argv[++i]);
      size_t sz = strtoull(argv[++i], 0, 10);
      uint64_t u0 = used();
      size_t d0 = dev_used();
      void** ps = (void**)calloc(n, sizeof(void*));
      int bad = 0;
      for (int k = 0; k < n; ++k) bad += hipMalloc(&ps[k], sz) != hipSuccess;
      uint64_t u1 = used();
      size_t d1 = dev_used();
      for (int k = 0; k < n; ++k) (void)hipFree(ps[k]);
      free(ps);
      printf("{\"op\":\"smalls\",\"count\":%d,\"size\":%zu,\"failed\":%d,\"shim_charge\":%llu,\"device_bytes\":%lld}\n",
             n, sz, bad, (unsigned long long)(u1 - u0), (long long)(d1 - d0));
    } else if (!strcmp(argv[i], "fill")) {
      // real HBM exhaustion (run WITHOUT the shim): leave about BYTES free
      size_t left = strtoull(argv[++i], 0, 10);
      size_t f = 0, t = 0, held = 0;
      for (int k = 0; k < 4096; ++k) {
        g_real_info(&f, &t);
        if (f <= left + (64u << 20)) break;
        size_t chunk = f - left > (8ull << 30) ? (8ull << 30) : (f - left) / 2;
        if (chunk < (32u << 20)) break;
        void* p = nullptr;
        if (hipMalloc(&p, chunk) != hipSuccess) break;
        held += chunk;
      }
      g_real_info(&f, &t);
      printf("{\"op\":\"fill\",\"held\":%zu,\"free\":%zu}\n", held, f);
    } else if (!strcmp(argv[i], "alloc")) {
      size_t n = strtoull(argv[++i], 0, 10);
      void* p = nullptr;
      int rc = hipMalloc(&p, n);
      printf("{\"op\":\"alloc\",\"n\":%zu,\"rc\":%d,\"used\":%llu,\"denied\":%llu}\n", n, rc,
             (unsigned long long)used(), (unsigned long long)denied());
    }
    fflush(stdout);
  }
  return 0;
}
