// Driver pages next to broker granules in one reserved range: the quota shim's VMM windows back
// 1 GiB slots with imported broker granules and, past the arena, map driver handles of the
// program's page size (or the part of a page in the next slot). On the real runtime (round 5,
// test_vmm_pages_come_from_the_arena[0.97]) hipMemSetAccess on such a driver page failed with
// hipErrorInvalidValue, at a different page from run to run. This probe takes the shim out of
// the picture and tries the same layouts directly, one case at a time:
//
//   plain      reserve 4 GiB, driver pages of 20 MiB from +0
//   split      the same pages starting at +1 GiB + 8 MiB after a 12 MiB piece at +1 GiB
//   imported   slot 0 holds an imported 1 GiB handle (export + import of an own hipMemCreate),
//              then driver pieces at +1 GiB as in "split"
//   overres    like "imported", in a range reserved 1 GiB larger and used from its 1 GiB-aligned part
//   both_rw    like "imported", with access set again on the whole slot 0 before the pieces
//   offset12   20 MiB pages from +12 MiB, nothing mapped before them
//
// When an access fails the probe tries, in order, and counts which one worked: the same call
// again ("retry"), after hipDeviceSynchronize ("sync"), and one call over everything mapped
// since the start of the case ("span"); then it checks the page reads back what was written.
// (Round 5, first run: plain and overres_plain pass; split, imported and overres fail the first
// page after a 12 MiB piece; both_rw fails the piece and passes the pages.)
//
//   g++ -std=c++17 -O1 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o tools/diag/build/vmm_spill_probe \
//       tools/diag/vmm_spill_probe.cpp -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {
constexpr size_t kGiB = 1ull << 30, kMiB = 1ull << 20;

hipMemAllocationProp prop(bool shareable) {
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof p);
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleType = shareable ? hipMemHandleTypePosixFileDescriptor : hipMemHandleTypeNone;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  return p;
}

hipError_t rw(void* va, size_t n) {
  hipMemAccessDesc d;
  std::memset(&d, 0, sizeof d);
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  return hipMemSetAccess(va, n, &d, 1);
}

struct Case {
  std::string name;
  std::string out;
  std::vector<hipMemGenericAllocationHandle_t> hs;
  std::vector<std::pair<char*, size_t>> maps;
  void* res = nullptr;
  size_t res_size = 0;
  char* first = nullptr;  // start of what the case mapped
  int fails = 0, retry_ok = 0, sync_ok = 0, span_ok = 0, readback_bad = 0;

  void rec(const char* k, long v) {
    char b[96];
    std::snprintf(b, sizeof b, "%s\"%s\": %ld", out.empty() ? "" : ", ", k, v);
    out += b;
  }
  // a driver handle of n bytes at va, access set; returns the first error
  int piece(char* va, size_t n) {
    auto p = prop(false);
    hipMemGenericAllocationHandle_t h = nullptr;
    hipError_t e = hipMemCreate(&h, n, &p, 0);
    if (e != hipSuccess) return 100 + e;
    hs.push_back(h);
    if ((e = hipMemMap(va, n, 0, h, 0)) != hipSuccess) return 200 + e;
    maps.push_back({va, n});
    if (!first) first = va;
    if ((e = rw(va, n)) != hipSuccess) {
      ++fails;
      (void)hipGetLastError();
      if (rw(va, n) == hipSuccess) {
        ++retry_ok;
      } else if ((void)hipDeviceSynchronize(), (void)hipGetLastError(), rw(va, n) == hipSuccess) {
        ++sync_ok;
      } else if ((void)hipGetLastError(), rw(first, size_t(va + n - first)) == hipSuccess) {
        ++span_ok;
      } else {
        (void)hipGetLastError();
        return 300 + e;
      }
    }
    if (hipMemset(va, 0x3c, n) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 400;
    unsigned char b[64];
    if (hipMemcpy(b, va + n - sizeof b, sizeof b, hipMemcpyDeviceToHost) != hipSuccess) return 500;
    for (unsigned char x : b) readback_bad += x != 0x3c;
    return 0;
  }
  void cleanup() {
    for (auto& m : maps) (void)hipMemUnmap(m.first, m.second);
    for (auto h : hs) (void)hipMemRelease(h);
    if (res) (void)hipMemAddressFree(res, res_size);
    (void)hipGetLastError();
  }
};

std::string run(const char* name, bool split, bool imported, bool overres, bool both_rw, size_t start_off = 0) {
  Case c;
  c.name = name;
  size_t want = 4 * kGiB;
  c.res_size = overres ? want + kGiB : want;
  if (hipMemAddressReserve(&c.res, c.res_size, overres ? 0 : kGiB, nullptr, 0) != hipSuccess) return "{\"reserve\": -1}";
  char* base = static_cast<char*>(c.res);
  c.rec("reserve_mod_gib_mib", long((reinterpret_cast<uintptr_t>(base) % kGiB) / kMiB));
  if (overres) base = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(base) + kGiB - 1) & ~uintptr_t(kGiB - 1));
  char* at = base + start_off;
  if (imported) {
    auto p = prop(true);
    hipMemGenericAllocationHandle_t h = nullptr, hi = nullptr;
    c.rec("create_1g", hipMemCreate(&h, kGiB, &p, 0));
    c.hs.push_back(h);
    int fd = -1;
    c.rec("export", hipMemExportToShareableHandle(&fd, h, hipMemHandleTypePosixFileDescriptor, 0));
    int rt = 0;
    (void)hipRuntimeGetVersion(&rt);
    hipError_t e = rt < 70100000 ? hipMemImportFromShareableHandle(&hi, &fd, hipMemHandleTypePosixFileDescriptor)
                                 : hipMemImportFromShareableHandle(
                                       &hi, reinterpret_cast<void*>(static_cast<intptr_t>(fd)),
                                       hipMemHandleTypePosixFileDescriptor);
    c.rec("import", e);
    c.hs.push_back(hi);
    c.rec("map_slot0", hipMemMap(base, kGiB, 0, hi, 0));
    c.maps.push_back({base, kGiB});
    c.rec("access_slot0", rw(base, kGiB));
    c.first = base;
    if (both_rw) c.rec("access_slot0_again", rw(base, kGiB));
    at = base + kGiB;
  }
  if (split) {
    c.rec("piece12", c.piece(at, 12 * kMiB));
    at += 12 * kMiB;
  }
  int failed_at = -1, err = 0;
  for (int k = 0; k < 40; ++k) {
    int r = c.piece(at + size_t(k) * 20 * kMiB, 20 * kMiB);
    if (r) {
      failed_at = k;
      err = r;
      break;
    }
  }
  c.rec("pages_failed_at", failed_at);
  c.rec("pages_err", err);
  c.rec("access_fails", c.fails);
  c.rec("retry_ok", c.retry_ok);
  c.rec("sync_ok", c.sync_ok);
  c.rec("span_ok", c.span_ok);
  c.rec("readback_bad", c.readback_bad);
  c.cleanup();
  return "\"" + c.name + "\": {" + c.out + "}";
}
}  // namespace

int main() {
  if (hipSetDevice(0) != hipSuccess) return 2;
  int rt = 0;
  (void)hipRuntimeGetVersion(&rt);
  std::string o = "{\"runtime_version\": " + std::to_string(rt);
  o += ", " + run("plain", false, false, false, false);
  o += ", " + run("split", true, false, false, false);
  o += ", " + run("imported", true, true, false, false);
  o += ", " + run("overres", true, true, true, false);
  o += ", " + run("both_rw", true, true, false, true);
  o += ", " + run("overres_plain", false, false, true, false);
  o += ", " + run("offset12", false, false, false, false, 12 * kMiB);
  o += ", " + run("split_again", true, false, false, false);
  std::puts((o + "}").c_str());
  return 0;
}
