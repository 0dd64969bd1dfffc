// Probe: how a queue CU mask maps onto the MI355X's XCDs / shader engines / CUs.
//
// For each mask, a stream is created with hipExtStreamCreateWithCUMask and a grid of short
// sleeping workgroups records where it ran (HW_REG_XCC_ID, HW_REG_HW_ID's SE/CU fields). The
// output says which mask bits select which XCD, i.e. how the plugin must build an XCD-aligned
// HSA_CU_MASK so a pod's CUs share one L2 and no other pod's. A compute-bound FMA kernel is timed
// per mask so the throughput-vs-CU-count line is measured, not assumed.
//
// hipcc --offload-arch=gfx950 -O2 tools/cu_mask_probe.hip -o cu_mask_probe && ./cu_mask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// s_getreg immediates: id | offset << 6 | (size - 1) << 11
constexpr int kHwId = 4 | (0 << 6) | (31 << 11);    // HW_REG_HW_ID (amd_device_functions.h: HW_ID)
constexpr int kXccId = 20 | (0 << 6) | (15 << 11);  // HW_REG_XCC_ID (gfx942/950)

__global__ void where(unsigned* out, int spin) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg(kHwId);
    unsigned xcc = __builtin_amdgcn_s_getreg(kXccId) & 0xf;
    out[blockIdx.x] = (xcc << 16) | (hw & 0xffff);
  }
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(127);
}

__global__ void burn(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.999f, d = blockIdx.x * 1e-4f;
  for (int i = 0; i < iters; ++i) {
    a = __builtin_fmaf(a, b, c);
    d = __builtin_fmaf(d, c, b);
    b = __builtin_fmaf(b, d, a) * 1e-7f + 1.0001f;
  }
  if (a + d == 12345.f) out[blockIdx.x] = b;
}

static std::string hexmask(const std::vector<uint32_t>& m) {
  std::string s = "0x";
  char buf[16];
  for (int i = (int)m.size() - 1; i >= 0; --i) {
    snprintf(buf, sizeof buf, "%08x", m[i]);
    s += buf;
  }
  return s;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const int words = (ncu + 31) / 32;
  printf("{\"device\": \"%s\", \"cus\": %d}\n", p.gcnArchName, ncu);

  struct Case {
    std::string name;
    std::vector<int> bits;
  };
  std::vector<Case> cases;
  auto range = [](int a, int b, int step = 1) {
    std::vector<int> v;
    for (int i = a; i < b; i += step) v.push_back(i);
    return v;
  };
  cases.push_back({"all", range(0, ncu)});
  for (int x = 0; x < 8; ++x) cases.push_back({"bit%8==" + std::to_string(x), range(x, ncu, 8)});
  for (int x = 0; x < 8; ++x) cases.push_back({"bits[" + std::to_string(32 * x) + ",+32)", range(32 * x, 32 * x + 32)});
  cases.push_back({"bits[0,128)", range(0, 128)});
  cases.push_back({"bit%8<4", {}});
  for (int i = 0; i < ncu; ++i)
    if (i % 8 < 4) cases.back().bits.push_back(i);
  cases.push_back({"bit0", {0}});
  cases.push_back({"bit1", {1}});
  cases.push_back({"bit8", {8}});

  const int nblk = 4096;
  unsigned* d_out;
  float* d_f;
  CHECK(hipMalloc(&d_out, nblk * sizeof(unsigned)));
  CHECK(hipMalloc(&d_f, 65536 * sizeof(float)));
  std::vector<unsigned> h(nblk);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));

  // argv[1] == "env": skip the per-stream masks (observed on the pool: the first ~6 masked
  // streams run on all 256 CUs, then stream creation stalls) and only report the default stream.
  const bool env_only = argc > 1 && std::string(argv[1]) == "env";
  for (auto& c : cases) {
    if (env_only) break;
    std::vector<uint32_t> m(words, 0);
    for (int b : c.bits) m[b / 32] |= 1u << (b % 32);
    hipStream_t s;
    CHECK(hipExtStreamCreateWithCUMask(&s, words, m.data()));
    CHECK(hipMemsetAsync(d_out, 0xff, nblk * sizeof(unsigned), s));
    hipLaunchKernelGGL(where, dim3(nblk), dim3(64), 0, s, d_out, 4);
    CHECK(hipMemcpyAsync(h.data(), d_out, nblk * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    CHECK(hipStreamSynchronize(s));
    std::set<std::tuple<int, int, int>> cus;       // (xcc, se, cu)
    std::map<int, std::set<std::pair<int, int>>> per_xcc;
    for (unsigned v : h) {
      int xcc = v >> 16, se = (v >> 13) & 3, cu = (v >> 8) & 15, sh = (v >> 12) & 1;
      cus.insert({xcc, se * 2 + sh, cu});
      per_xcc[xcc].insert({se * 2 + sh, cu});
    }
    // throughput: 8 x #CU blocks of 256 threads, FMA-bound
    const int tb = 8 * ncu, iters = 20000;
    hipLaunchKernelGGL(burn, dim3(tb), dim3(256), 0, s, d_f, iters);
    CHECK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(burn, dim3(tb), dim3(256), 0, s, d_f, iters);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"case\": \"%s\", \"mask\": \"%s\", \"bits\": %zu, \"distinct_cus\": %zu, \"per_xcc\": {",
           c.name.c_str(), hexmask(m).c_str(), c.bits.size(), cus.size());
    bool first = true;
    for (auto& [x, set] : per_xcc) {
      printf("%s\"%d\": %zu", first ? "" : ", ", x, set.size());
      first = false;
    }
    printf("}, \"burn_ms\": %.3f}\n", ms);
    fflush(stdout);
    CHECK(hipStreamDestroy(s));
  }
  // Optional: where does a default stream run (shows HSA_CU_MASK / ROC_GLOBAL_CU_MASK effect).
  {
    CHECK(hipMemset(d_out, 0xff, nblk * sizeof(unsigned)));
    hipLaunchKernelGGL(where, dim3(nblk), dim3(64), 0, 0, d_out, 4);
    CHECK(hipMemcpy(h.data(), d_out, nblk * sizeof(unsigned), hipMemcpyDeviceToHost));
    std::set<std::tuple<int, int, int>> cus;
    std::map<int, int> per_xcc;
    for (unsigned v : h) {
      int xcc = v >> 16, se = (v >> 13) & 3, cu = (v >> 8) & 15, sh = (v >> 12) & 1;
      if (cus.insert({xcc, se * 2 + sh, cu}).second) per_xcc[xcc]++;
    }
    const int tb = 8 * ncu, iters = 20000;
    hipLaunchKernelGGL(burn, dim3(tb), dim3(256), 0, 0, d_f, iters);
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(burn, dim3(tb), dim3(256), 0, 0, d_f, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const char* env1 = getenv("HSA_CU_MASK");
    const char* env2 = getenv("ROC_GLOBAL_CU_MASK");
    printf("{\"case\": \"default-stream\", \"HSA_CU_MASK\": \"%s\", \"ROC_GLOBAL_CU_MASK\": \"%s\", \"distinct_cus\": %zu, \"per_xcc\": {",
           env1 ? env1 : "", env2 ? env2 : "", cus.size());
    bool first = true;
    for (auto& [x, n] : per_xcc) {
      printf("%s\"%d\": %d", first ? "" : ", ", x, n);
      first = false;
    }
    printf("}, \"burn_ms\": %.3f}\n", ms);
  }
  CHECK(hipFree(d_out));
  CHECK(hipFree(d_f));
  return 0;
}
