// Probe for the isolating HBM broker of docs/HBM_TURNOVER.md.
//
// The broker holds the GPU's shareable HBM as VMM physical handles (hipMemCreate), one per
// granule, and exports each as a file descriptor. A tenant receives ONLY its granules' fds over a
// Unix socket (SCM_RIGHTS), imports them and maps them contiguously into its own address range:
// no tenant can reach another tenant's granules. When the tenant's connection closes, the broker
// zeroes the granules through its own mapping and hands them to the next tenant. No VRAM goes
// back to amdgpu, so nothing waits for the driver's wipe.
//
//   vmm_broker_probe broker <sock> <granules> <granule_mib> <tenants>
//   vmm_broker_probe tenant <sock>
//
// Each side prints JSON lines; tools/diag/vmm_broker_probe.py drives both as child processes.
#include <hip/hip_runtime.h>

#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("{\"error\": \"%s\", \"at\": \"%s\"}\n", hipGetErrorString(e_), #x); \
      std::fflush(stdout);                                                            \
      std::exit(3);                                                                   \
    }                                                                                 \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

static hipMemAllocationProp device_prop() {
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof p);
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  return p;
}

static hipMemAccessDesc rw_access() {
  hipMemAccessDesc d;
  std::memset(&d, 0, sizeof d);
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  return d;
}

// header {count, granule bytes} then the fds, at most 200 per message
static bool send_fds(int s, const std::vector<int>& fds, size_t gran) {
  unsigned long long hdr[2] = {fds.size(), gran};
  if (send(s, hdr, sizeof hdr, 0) != (ssize_t)sizeof hdr) return false;
  for (size_t i = 0; i < fds.size(); i += 200) {
    size_t n = std::min<size_t>(200, fds.size() - i);
    char byte = 'f';
    iovec io{&byte, 1};
    std::vector<char> ctl(CMSG_SPACE(n * sizeof(int)));
    msghdr m{};
    m.msg_iov = &io;
    m.msg_iovlen = 1;
    m.msg_control = ctl.data();
    m.msg_controllen = ctl.size();
    cmsghdr* c = CMSG_FIRSTHDR(&m);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(n * sizeof(int));
    std::memcpy(CMSG_DATA(c), fds.data() + i, n * sizeof(int));
    if (sendmsg(s, &m, 0) != 1) return false;
  }
  return true;
}

static bool recv_fds(int s, std::vector<int>& fds, size_t& gran) {
  unsigned long long hdr[2];
  if (recv(s, hdr, sizeof hdr, MSG_WAITALL) != (ssize_t)sizeof hdr) return false;
  gran = hdr[1];
  while (fds.size() < hdr[0]) {
    size_t n = std::min<size_t>(200, hdr[0] - fds.size());
    char byte;
    iovec io{&byte, 1};
    std::vector<char> ctl(CMSG_SPACE(n * sizeof(int)));
    msghdr m{};
    m.msg_iov = &io;
    m.msg_iovlen = 1;
    m.msg_control = ctl.data();
    m.msg_controllen = ctl.size();
    if (recvmsg(s, &m, 0) != 1) return false;
    cmsghdr* c = CMSG_FIRSTHDR(&m);
    if (!c || c->cmsg_type != SCM_RIGHTS) return false;
    size_t got = (c->cmsg_len - CMSG_LEN(0)) / sizeof(int);
    const int* p = reinterpret_cast<const int*>(CMSG_DATA(c));
    fds.insert(fds.end(), p, p + got);
  }
  return true;
}

static int broker(const char* path, int granules, size_t gran_mib, int tenants) {
  CK(hipSetDevice(0));
  hipMemAllocationProp prop = device_prop();
  size_t min_gran = 0;
  CK(hipMemGetAllocationGranularity(&min_gran, &prop, hipMemAllocationGranularityMinimum));
  size_t gran = gran_mib << 20;
  if (gran % min_gran) {
    std::printf("{\"error\": \"granule not a multiple of %zu\"}\n", min_gran);
    return 2;
  }
  double t0 = now_ms();
  std::vector<hipMemGenericAllocationHandle_t> h(granules);
  std::vector<int> fds(granules);
  for (int i = 0; i < granules; ++i) {
    CK(hipMemCreate(&h[i], gran, &prop, 0));
    int fd = -1;
    CK(hipMemExportToShareableHandle(&fd, h[i], hipMemHandleTypePosixFileDescriptor, 0));
    fds[i] = fd;
  }
  size_t total = gran * granules;
  void* base = nullptr;
  CK(hipMemAddressReserve(&base, total, 0, nullptr, 0));
  for (int i = 0; i < granules; ++i)
    CK(hipMemMap(static_cast<char*>(base) + i * gran, gran, 0, h[i], 0));
  hipMemAccessDesc acc = rw_access();
  CK(hipMemSetAccess(base, total, &acc, 1));
  CK(hipMemset(base, 0, total));
  CK(hipDeviceSynchronize());
  double t1 = now_ms();

  int ls = socket(AF_UNIX, SOCK_STREAM, 0);
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  std::snprintf(a.sun_path, sizeof a.sun_path, "%s", path);
  unlink(path);
  if (bind(ls, (sockaddr*)&a, sizeof a) || listen(ls, 4)) {
    std::printf("{\"error\": \"bind %s\"}\n", path);
    return 2;
  }
  std::printf("{\"broker_ready\": true, \"granules\": %d, \"granule_mib\": %zu, "
              "\"min_granularity\": %zu, \"setup_ms\": %.1f}\n",
              granules, gran_mib, min_gran, t1 - t0);
  std::fflush(stdout);
  for (int k = 0; k < tenants; ++k) {
    int c = accept(ls, nullptr, nullptr);
    if (c < 0) return 2;
    double ts = now_ms();
    if (!send_fds(c, fds, gran)) {
      std::printf("{\"error\": \"send_fds\"}\n");
      return 2;
    }
    double tsent = now_ms();
    char buf[64];
    while (recv(c, buf, sizeof buf, 0) > 0) {
    }  // the tenant is gone when its end closes (exit or crash)
    close(c);
    double tg = now_ms();
    CK(hipMemset(base, 0, total));  // scrub before the next tenant
    CK(hipDeviceSynchronize());
    double tz = now_ms();
    std::printf("{\"tenant\": %d, \"send_ms\": %.2f, \"scrub_ms\": %.2f, \"scrub_GBps\": %.0f, "
                "\"held_ms\": %.1f}\n",
                k, tsent - ts, tz - tg, total / ((tz - tg) / 1e3) / 1e9, tg - ts);
    std::fflush(stdout);
  }
  close(ls);
  unlink(path);
  CK(hipMemUnmap(base, total));
  CK(hipMemAddressFree(base, total));
  for (int i = 0; i < granules; ++i) {
    close(fds[i]);
    CK(hipMemRelease(h[i]));
  }
  return 0;
}

static int tenant(const char* path) {
  double t0 = now_ms();
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  double t1 = now_ms();
  int s = socket(AF_UNIX, SOCK_STREAM, 0);
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  std::snprintf(a.sun_path, sizeof a.sun_path, "%s", path);
  if (connect(s, (sockaddr*)&a, sizeof a)) {
    std::printf("{\"error\": \"connect\"}\n");
    return 2;
  }
  std::vector<int> fds;
  size_t gran = 0;
  if (!recv_fds(s, fds, gran)) {
    std::printf("{\"error\": \"recv_fds\"}\n");
    return 2;
  }
  double t2 = now_ms();
  size_t total = gran * fds.size();
  std::vector<hipMemGenericAllocationHandle_t> h(fds.size());
  // VMM_IMPORT_BY_PTR=1: pass the address of the fd (what some HIP releases dereference)
  const bool by_ptr = getenv("VMM_IMPORT_BY_PTR") && getenv("VMM_IMPORT_BY_PTR")[0] == '1';
  int rtv = 0;
  CK(hipRuntimeGetVersion(&rtv));
  for (size_t i = 0; i < fds.size(); ++i)
    CK(hipMemImportFromShareableHandle(&h[i],
                                       by_ptr ? static_cast<void*>(&fds[i])
                                              : reinterpret_cast<void*>(static_cast<intptr_t>(fds[i])),
                                       hipMemHandleTypePosixFileDescriptor));
  double t3 = now_ms();
  void* base = nullptr;
  CK(hipMemAddressReserve(&base, total, 0, nullptr, 0));
  for (size_t i = 0; i < fds.size(); ++i)
    CK(hipMemMap(static_cast<char*>(base) + i * gran, gran, 0, h[i], 0));
  hipMemAccessDesc acc = rw_access();
  CK(hipMemSetAccess(base, total, &acc, 1));
  double t4 = now_ms();
  // the broker scrubbed it: sample one byte per granule before writing
  unsigned nonzero = 0;
  for (size_t i = 0; i < fds.size(); ++i) {
    unsigned char b = 1;
    CK(hipMemcpy(&b, static_cast<char*>(base) + i * gran + gran / 2, 1, hipMemcpyDeviceToHost));
    nonzero += b != 0;
  }
  double t5 = now_ms();
  CK(hipMemset(base, 7, total));
  CK(hipDeviceSynchronize());
  double t6 = now_ms();
  std::printf("{\"runtime_version\": %d, \"by_ptr\": %d, \"tenant_gib\": %.1f, \"hip_init_ms\": %.1f, \"recv_ms\": %.2f, \"import_ms\": %.2f, "
              "\"map_ms\": %.2f, \"write_ms\": %.1f, \"write_GBps\": %.0f, "
              "\"nonzero_granules_seen\": %u, \"ready_ms\": %.1f}\n",
              rtv, int(by_ptr), total / double(1ull << 30), t1 - t0, t2 - t1, t3 - t2, t4 - t3, t6 - t5,
              total / ((t6 - t5) / 1e3) / 1e9, nonzero, (t4 - t1));
  std::fflush(stdout);
  return 0;  // exit: the mappings go with the process, the broker's handles keep the memory
}

int main(int argc, char** argv) {
  if (argc >= 6 && !std::strcmp(argv[1], "broker"))
    return broker(argv[2], std::atoi(argv[3]), std::strtoull(argv[4], nullptr, 10), std::atoi(argv[5]));
  if (argc >= 3 && !std::strcmp(argv[1], "tenant")) return tenant(argv[2]);
  std::fprintf(stderr, "usage: %s broker <sock> <granules> <granule_mib> <tenants> | tenant <sock>\n",
               argv[0]);
  return 2;
}
