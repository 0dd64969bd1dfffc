// vmm_tenant: a pod process that allocates the way PyTorch's expandable segments do (one large
// reserved VA range, fixed-size pages created and mapped one after another, access set per
// mapped run), on the real HIP runtime. Under the quota shim with an HBM broker grant the pages
// come from the arena (quota/hbmbroker.py, native/hipshim "VMM from the arena");
// tests/test_hbm_broker.py runs it on MI355X.
//
//   vmm_tenant <fill fraction of the quota> [page MiB = 20]
//
// It fills `fill` of the device total it is shown (the quota under the shim), writes every page
// with its own byte and reads each back, unmaps every other page of the first half and maps new
// pages into the holes (the segment shrinking and growing), checks again, and prints one JSON
// line; then it unmaps everything, frees the range and prints a second line.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {
struct Page {
  char* va;
  hipMemGenericAllocationHandle_t h;
};

bool check(hipError_t e, const char* what) {
  if (e != hipSuccess) std::fprintf(stderr, "vmm_tenant: %s: %s\n", what, hipGetErrorString(e));
  return e == hipSuccess;
}

template <class F>
F shim(const char* n) {
  return reinterpret_cast<F>(dlsym(RTLD_DEFAULT, n));
}

void stats(char* out, size_t cap) {
  uint64_t v[5] = {0}, u[4] = {0}, a[2] = {0};
  int w = -1, on = -1;
  if (auto f = shim<int (*)(uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*)>("gpushare_shim_vmm_stats"))
    w = f(&v[0], &v[1], &v[2], &v[3], &v[4]);
  if (auto f = shim<int (*)(uint64_t*, uint64_t*, uint64_t*, uint64_t*)>("gpushare_shim_stats")) f(&u[0], &u[1], &u[2], &u[3]);
  if (auto f = shim<int (*)(uint64_t*, uint64_t*)>("gpushare_shim_arena_stats")) on = f(&a[0], &a[1]);
  std::snprintf(out, cap,
                "\"windows\": %d, \"vmm_creates\": %llu, \"arena_maps\": %llu, \"real_pieces\": %llu, "
                "\"slots_backed\": %llu, \"slots_now\": %llu, \"ledger_used\": %llu, \"quota\": %llu, \"denied\": %llu, "
                "\"arena\": %d, \"arena_size\": %llu, \"arena_used\": %llu",
                w, (unsigned long long)v[0], (unsigned long long)v[1], (unsigned long long)v[2], (unsigned long long)v[3],
                (unsigned long long)v[4], (unsigned long long)u[0], (unsigned long long)u[1], (unsigned long long)u[2], on,
                (unsigned long long)a[0], (unsigned long long)a[1]);
}

bool fill_and_check(const std::vector<Page>& pages, size_t page, int salt) {
  std::vector<unsigned char> host(4096);
  for (size_t k = 0; k < pages.size(); ++k)
    if (!check(hipMemset(pages[k].va, int((k + salt) & 0xff), page), "hipMemset")) return false;
  if (!check(hipDeviceSynchronize(), "sync")) return false;
  for (size_t k = 0; k < pages.size(); ++k)
    for (size_t off : {size_t(0), page - 4096}) {
      if (!check(hipMemcpy(host.data(), pages[k].va + off, 4096, hipMemcpyDeviceToHost), "hipMemcpy")) return false;
      for (unsigned char c : host)
        if (c != ((k + salt) & 0xff)) return false;
    }
  return true;
}
}  // namespace

int main(int argc, char** argv) {
  double fill = argc > 1 ? std::atof(argv[1]) : 0.85;
  size_t page = (argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 20) << 20;
  if (!check(hipSetDevice(0), "hipSetDevice")) return 2;
  hipDeviceProp_t prop;
  if (!check(hipGetDeviceProperties(&prop, 0), "hipGetDeviceProperties")) return 2;
  size_t total = prop.totalGlobalMem;  // the quota, under the shim
  size_t range = (total + total / 8 + page - 1) / page * page;
  void* base = nullptr;
  if (!check(hipMemAddressReserve(&base, range, 0, nullptr, 0), "hipMemAddressReserve")) return 2;
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof p);
  p.type = hipMemAllocationTypePinned;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  hipMemAccessDesc acc;
  std::memset(&acc, 0, sizeof acc);
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = 0;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  std::vector<Page> pages;
  size_t want = size_t(double(total) * fill) / page;
  int create_err = 0, map_err = 0, access_err = 0;
  long fail_page = -1;
  for (size_t k = 0; k < want; ++k) {
    Page pg{static_cast<char*>(base) + k * page, nullptr};
    hipError_t e = hipMemCreate(&pg.h, page, &p, 0);
    if (e != hipSuccess) {
      create_err = e;
      break;
    }
    e = hipMemMap(pg.va, page, 0, pg.h, 0);
    if (e != hipSuccess) {
      map_err = e;
    } else if ((e = hipMemSetAccess(pg.va, page, &acc, 1)) != hipSuccess) {
      access_err = e;
      (void)hipMemUnmap(pg.va, page);
    }
    if (e != hipSuccess) {
      fail_page = long(k);
      (void)hipMemRelease(pg.h);
      break;
    }
    pages.push_back(pg);
  }
  bool ok1 = !pages.empty() && fill_and_check(pages, page, 1);
  // shrink and grow: every other page of the first half leaves, new pages fill the holes
  size_t holes = 0;
  for (size_t k = 0; k < pages.size() / 2; k += 2) {
    ok1 = ok1 && check(hipMemUnmap(pages[k].va, page), "hipMemUnmap") && check(hipMemRelease(pages[k].h), "hipMemRelease");
    pages[k].h = nullptr;
    ++holes;
  }
  bool ok2 = ok1;
  for (size_t k = 0; k < pages.size() / 2 && ok2; k += 2) {
    ok2 = check(hipMemCreate(&pages[k].h, page, &p, 0), "hipMemCreate (refill)") &&
          check(hipMemMap(pages[k].va, page, 0, pages[k].h, 0), "hipMemMap (refill)") &&
          check(hipMemSetAccess(pages[k].va, page, &acc, 1), "hipMemSetAccess (refill)");
  }
  ok2 = ok2 && fill_and_check(pages, page, 7);
  char st[1024];
  stats(st, sizeof st);
  std::printf("{\"phase\": \"filled\", \"total\": %zu, \"page\": %zu, \"pages\": %zu, \"want\": %zu, \"bytes\": %zu, "
              "\"create_err\": %d, \"map_err\": %d, \"access_err\": %d, \"fail_page\": %ld, \"base_mod_gib\": %zu, "
              "\"holes\": %zu, \"ok_fill\": %s, \"ok_refill\": %s, %s}\n",
              total, page, pages.size(), want, pages.size() * page, create_err, map_err, access_err, fail_page,
              size_t(reinterpret_cast<uintptr_t>(base) % (1ull << 30)), holes, ok1 ? "true" : "false",
              ok2 ? "true" : "false", st);
  std::fflush(stdout);
  for (auto& pg : pages)
    if (pg.h) {
      (void)hipMemUnmap(pg.va, page);
      (void)hipMemRelease(pg.h);
    }
  (void)hipMemAddressFree(base, range);
  stats(st, sizeof st);
  std::printf("{\"phase\": \"released\", %s}\n", st);
  return ok1 && ok2 ? 0 : 1;
}
