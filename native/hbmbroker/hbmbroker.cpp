// gpushare-hbm-broker: one per GPU. Holds the GPU's shareable HBM as VMM physical handles, one per
// granule (hipMemCreate, exported as dma-buf fds), and lends granules to pods.
//
// Why: amdgpu wipes every VRAM buffer a process frees before it hands the memory out again, on
// SDMA at ~33 GB/s per GPU (docs/HBM_TURNOVER.md). A replacement pod therefore waits seconds for
// a retired pod's HBM. The broker never frees: when a pod is gone it zeroes the pod's granules
// through its own mapping (hipMemsetAsync, ~6 TB/s) and lends them to the next pod.
//
// Isolation: a pod receives ONLY the fds of its own granules (SCM_RIGHTS) and maps them into its
// own address space; it cannot name another pod's granules. The amount is set by the granter
// (the device plugin) on an admin socket that lives outside every directory mounted into a
// container (mode 0600, and the peer's SO_PEERCRED uid must be the broker's or root); a pod takes
// its grant with its token (again after a container restart).
//
// Protocol: one text line per request.
//   admin socket (--admin-socket, 0600):
//     "GRANT <token> <bytes> [<limit bytes>]\n" -> "OK <granules>\n" | "ERR ...\n" (a repeated
//                                  grant refreshes it). <limit>: the pod's whole quota; it may
//                                  borrow granules beyond its grant up to that (EXTEND below)
//     "REVOKE <token>\n"        -> "OK <held>\n": the token can never be taken again; a process
//                                  holding it keeps its granules until its connection ends, and
//                                  is sent "END\n" (no more granules)
//     "SIZE <granules>|max\n"   -> "OK <granules> <target>\n": how much of the GPU the broker may
//                                  hold. Free granules beyond it go back to the driver at once,
//                                  lent ones when they come back; below it the broker grows as the
//                                  driver has room (SIZE 0: a cgpu.disable.isolation node)
//     "LIST\n"                  -> one JSON line {"boot": .., "grants": {token: granules, ..}}
//     "STAT\n"                  -> one JSON line of counters, with this process's "boot" id
//   pod socket (--socket, 0666):
//     "TAKE <token>\n"          -> "FDS <n> <granule bytes>\n", then n fds (batches of <= 200,
//                                  one byte each); the connection stays open: its end (close,
//                                  exit, crash) returns the granules, which are scrubbed first.
//     "TAKE <token> STREAM\n"   -> "FDS <k> <granule bytes> <n> <limit>\n" + k fds at once (k =
//                                  what is free now, possibly 0), then "MORE <j> <granule bytes>\n"
//                                  + j fds as granules come back, until all n are delivered: the
//                                  pod maps the first granules while a retiring pod's are still
//                                  being torn down, instead of waiting for all n. Owed granules
//                                  that have not come within --wait-s are cancelled with "END\n".
//     after a TAKE was served and nothing is owed:
//     "EXTEND <k>\n"            -> "XFDS <j> <granule bytes>\n" + j fds, j <= k: granules beyond
//                                  the grant, up to the grant's limit, from granules no grant
//                                  has a claim on (j = 0 when there are none: the pod uses the
//                                  driver). They return with the connection like the others.
//     "AVAIL\n"                 -> "AVAIL <j>\n": what EXTEND could give now (hipMemGetInfo)
// A TAKE whose granules are still held by a retiring pod waits (up to --wait-s), and one whose
// grant has not arrived yet waits up to --ungranted-wait-s (a broker that just restarted is
// re-granted by the plugin within a poll interval): the pod's runtime may start before the
// retired pod is gone, or before the plugin has seen this broker, as on a booting node.
//
// Sizing: the broker is sized for the GPU less --reserve-gib (the pods' runtimes, and whatever
// of their quota is not lent as granules, come from the driver). Every pod can use its whole
// quota: its grant (a share of the quota) is lent at once, granules no grant claims can be
// borrowed beyond it (EXTEND), and the driver serves the rest. Free granules are given back to the
// driver when its free memory drops under --low-water-gib (default half the reserve), and the
// broker grows again once the driver has more than the reserve free.
//
// The boot id changes with every start. The plugin polls STAT, and on a new boot id it re-grants
// every live pod's token: a broker restart loses no grant that a pod still needs.
//
// Scrubs are asynchronous: a released pod's granules are zeroed on the broker's stream by its
// scrub kernel (scrub.hip: non-temporal 16 B stores; hipMemsetAsync if the code object is
// missing), in chunks of --scrub-chunk granules with an event each, and each chunk is lent again
// once its event has completed. GRANT, TAKE and STAT are served while the GPU zeroes.
//
// Release policy (--release-policy): before a released granule is lent again, "refs" waits until
// no reference to its dma-buf is left outside the broker (fdinfo "count:"), "exit" waits until
// the holding process has exited (pidfd), "trust" lends it at once (tests only). The default
// "auto" is refs where the kernel reports the count, else exit.
//
//   gpushare-hbm-broker --socket /run/gpushare/hbm/gpu0/hbm0.sock
//                       --admin-socket /run/gpushare/hbm/admin/hbm0.sock
//                       [--device 0 | --pci-bus-id 0000:05:00.0] [--gib N | --reserve-gib R]
//                       [--granule-mib 1024] [--wait-s 30] [--ungranted-wait-s 10]
//                       [--grant-ttl-s 0] [--max-clients 1024] [--max-per-peer 8]
//                       [--request-timeout-s 2] [--release-policy auto] [--scrub-chunk 8]
//                       [--scrub-kernel <dir of this executable>/gpushare-hbm-scrub.co]
//                       [--start-empty] [--low-water-gib R/2]
// --start-empty: hold nothing until the granter sends SIZE (the DaemonSet: the plugin knows
// whether the node is cgpu-disabled, the broker does not).
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void die(const char* what, hipError_t e) {
  std::fprintf(stderr, "gpushare-hbm-broker: %s: %s\n", what, hipGetErrorString(e));
  std::exit(3);
}

#define CK(x)                      \
  do {                             \
    hipError_t e_ = (x);           \
    if (e_ != hipSuccess) die(#x, e_); \
  } while (0)

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

int listen_unix(const std::string& path, mode_t mode) {
  int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  if (path.size() >= sizeof a.sun_path) {
    std::fprintf(stderr, "gpushare-hbm-broker: socket path too long: %s\n", path.c_str());
    std::exit(2);
  }
  std::memcpy(a.sun_path, path.c_str(), path.size() + 1);
  unlink(path.c_str());
  // created with the final mode: no window in which the admin socket is open to everyone
  mode_t old = umask(0777 & ~mode);
  int rc = bind(s, reinterpret_cast<sockaddr*>(&a), sizeof a);
  umask(old);
  if (rc || listen(s, 128)) {
    std::perror(path.c_str());
    std::exit(2);
  }
  chmod(path.c_str(), mode);
  return s;
}

std::string boot_id() {
  unsigned char b[8] = {0};
  int fd = open("/dev/urandom", O_RDONLY | O_CLOEXEC);
  if (fd < 0 || read(fd, b, sizeof b) != ssize_t(sizeof b)) {
    uint64_t t = uint64_t(now_s() * 1e9) ^ (uint64_t(getpid()) << 40);
    std::memcpy(b, &t, sizeof b);
  }
  if (fd >= 0) close(fd);
  char s[17];
  for (int i = 0; i < 8; ++i) std::snprintf(s + 2 * i, 3, "%02x", b[i]);
  return s;
}

int pidfd_of(pid_t pid) {
#ifdef SYS_pidfd_open
  if (pid > 0) return int(syscall(SYS_pidfd_open, pid, 0));
#endif
  (void)pid;
  return -1;
}

bool exited(int pidfd) {  // a pidfd polls readable once its process has exited
  pollfd p{pidfd, POLLIN, 0};
  return poll(&p, 1, 0) > 0;
}

bool valid_token(const char* t) {
  size_t n = std::strlen(t);
  if (n == 0 || n > 128) return false;
  for (size_t i = 0; i < n; ++i) {
    char c = t[i];
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '-' || c == '_'))
      return false;
  }
  return true;
}

struct Client {
  int fd = -1;
  bool admin = false;
  std::string in;
  double since = 0;       // connected at
  bool asked = false;     // a complete request line has arrived
  pid_t pid = 0;          // SO_PEERCRED (0: the peer is in another PID namespace)
  uid_t uid = 0;
  int pidfd = -1;         // release policy "exit": the holder's process, opened at its TAKE
  // a pod: the granules it holds (indices), or the token it waits for
  std::vector<int> held;
  std::string token;      // the grant it holds
  std::string waiting;    // token of a TAKE not yet served
  double wait_since = 0;
  bool stream = false;    // TAKE ... STREAM: granules are delivered as they become free
  int owed = 0;           // granules of its grant still to deliver (stream)
  int extra = 0;          // granules borrowed beyond the grant (EXTEND), part of `held`
};

enum Policy { kRefs, kExit, kTrust };

struct Broker {
  int device = 0;
  size_t gran = 1ull << 30;
  int count = 0;
  double wait_s = 30.0, ungranted_wait_s = 10.0, request_timeout_s = 2.0;
  size_t max_clients = 1024, max_per_peer = 8;
  Policy policy = kRefs;
  std::string boot = boot_id();
  std::vector<hipMemGenericAllocationHandle_t> h;
  std::vector<int> fds;
  // each granule mapped at an address range of its own, for the scrub: HIP gives a released
  // handle's memory back to the driver only once the range it was mapped in is freed too
  // (tools/diag/release_probe.cpp), so a granule going back frees its range
  std::vector<char*> va;
  hipStream_t stream = nullptr;
  std::deque<int> free_list;
  // released granules being zeroed: lent again once their event has completed
  struct Scrub {
    std::vector<int> idx;
    hipEvent_t ev;
    double t0;
  };
  std::deque<Scrub> scrubbing;
  // granules not lent again until their holder is really gone (see the release policy); one
  // release's granules go together
  struct Held {
    std::vector<int> idx;
    int pidfd = -1;  // kExit: the holder's process
    double t0 = 0;   // released at
  };
  std::vector<Held> quarantine;
  unsigned long long quarantined_total = 0, lost = 0;
  double quarantine_s_last = 0, quarantine_s_max = 0;  // release -> the last reference gone
  std::vector<int> base_refs;  // each granule's references with no tenant (the broker's own export)
  // A grant belongs to the pod, not to one process: a TAKE holds it while its connection lives,
  // and a restarted container (same env, same token) takes it again once the old process's
  // granules are back. It lives until the plugin revokes it (or grant_ttl_s after it was
  // granted or last released, when a TTL is set).
  struct Grant {
    int granules;
    int limit;        // granules it may hold with what it borrows (EXTEND): the pod's quota
    double at;
    int holder = -1;  // fd of the connection holding it
  };
  std::map<std::string, Grant> grants;
  std::set<std::string> revoked;
  std::deque<std::string> revoked_order;  // bounded: the oldest revocations are forgotten
  double grant_ttl_s = 0.0;
  int scrub_chunk = 8;  // granules per scrub event
  unsigned long long expired = 0;
  std::map<int, Client> clients;
  // stats
  unsigned long long takes = 0, releases = 0, refused = 0, timeouts = 0, busy = 0, idle_dropped = 0,
                     revokes = 0, peer_refused = 0, streamed = 0, more_msgs = 0;
  double scrub_s_total = 0, scrub_s_last = 0, setup_s = 0;
  // where the event loop's time goes: the longest pass, a release's bookkeeping, enqueueing a
  // scrub, and how long TAKEs waited to be answered
  double loop_s_max = 0, release_s_max = 0, scrub_enqueue_s_max = 0, take_wait_s_last = 0, take_wait_s_max = 0;
  double send_s_max = 0, last_send_at = 0;  // sending a batch of fds; wall clock of the last one
  unsigned long long scrubbed_bytes = 0;

  hipMemAllocationProp prop_{};
  // the scrub kernel (scrub.hip, a code object next to the executable): zeroes at HBM write
  // bandwidth with non-temporal stores; hipMemsetAsync when it is not there
  hipModule_t scrub_mod = nullptr;
  hipFunction_t scrub_fn = nullptr;
  hipFunction_t scrub_n_fn = nullptr;  // gs_scrub_n: up to 8 ranges in one dispatch
  unsigned long long scrub_dispatches = 0;
  std::string scrub_path;
  int count_max = 0;          // granules the broker is sized for (its address range)
  int target = 0;             // granules it may hold now (SIZE; count_max unless told otherwise)
  std::vector<char> present;  // granule i exists (created, exported, mapped)
  size_t reserve_bytes = 0;   // what it leaves to the driver
  size_t low_water_bytes = 0; // driver free memory under which free granules go back to it
  double last_pressure = 0;
  unsigned long long grown = 0, given_back = 0, pressure_given = 0, extends = 0, extended = 0, ends = 0;
  int counted = -1;           // the kernel reports dma-buf references in fdinfo: 1 yes, 0 no, -1 not known yet
  bool policy_auto = true;    // --release-policy auto: refs where counted, else exit

  hipMemAccessDesc rw() const {
    hipMemAccessDesc d;
    std::memset(&d, 0, sizeof d);
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = device;
    d.flags = hipMemAccessFlagsProtReadWrite;
    return d;
  }

  void load_scrub_kernel() {
    if (scrub_path.empty() || access(scrub_path.c_str(), R_OK) != 0) return;
    if (hipModuleLoad(&scrub_mod, scrub_path.c_str()) != hipSuccess ||
        hipModuleGetFunction(&scrub_fn, scrub_mod, "gs_scrub") != hipSuccess) {
      scrub_fn = nullptr;
      (void)hipGetLastError();
      std::fprintf(stderr, "gpushare-hbm-broker: scrub kernel %s not loaded: zeroing with hipMemsetAsync\n",
                   scrub_path.c_str());
      return;
    }
    if (hipModuleGetFunction(&scrub_n_fn, scrub_mod, "gs_scrub_n") != hipSuccess) {
      scrub_n_fn = nullptr;  // an older code object: one dispatch per range
      (void)hipGetLastError();
    }
  }

  // the kernel argument of gs_scrub_n (scrub.hip ScrubSet)
  struct ScrubSet {
    void* p[8];
    uint64_t n16[8];
    uint32_t count;
  };

  // zero [p, p + bytes) on the broker's stream
  void zero(char* p, size_t bytes) {
    if (scrub_fn && bytes % 16 == 0 && reinterpret_cast<uintptr_t>(p) % 16 == 0) {
      uint64_t n16 = bytes / 16;
      uint64_t blocks = std::min<uint64_t>(2048, (n16 + 255) / 256);  // 8 blocks of 4 waves per CU
      void* args[] = {&p, &n16};
      CK(hipModuleLaunchKernel(scrub_fn, unsigned(blocks), 1, 1, 256, 1, 1, 0, stream, args, nullptr));
      ++scrub_dispatches;
      return;
    }
    CK(hipMemsetAsync(p, 0, bytes, stream));
    ++scrub_dispatches;
  }

  // zero up to 8 ranges in one dispatch (gs_scrub_n), or one by one without it
  void zero_ranges(char* const* p, const size_t* bytes, int count) {
    bool ok = scrub_n_fn != nullptr && count > 1;
    for (int k = 0; ok && k < count; ++k)
      ok = bytes[k] % 16 == 0 && reinterpret_cast<uintptr_t>(p[k]) % 16 == 0;
    if (!ok) {
      for (int k = 0; k < count; ++k) zero(p[k], bytes[k]);
      return;
    }
    ScrubSet s;
    std::memset(&s, 0, sizeof s);
    s.count = uint32_t(count);
    for (int k = 0; k < count; ++k) s.p[k] = p[k], s.n16[k] = bytes[k] / 16;
    unsigned blocks = 2048u / unsigned(count) * unsigned(count);  // a multiple of count: blocks per range equal
    void* args[] = {&s};
    CK(hipModuleLaunchKernel(scrub_n_fn, blocks, 1, 1, 256, 1, 1, 0, stream, args, nullptr));
    ++scrub_dispatches;
  }

  // granule i: created, exported, mapped at a range of its own, readable and writable (not yet
  // zeroed). False (nothing held) when the device has no room for it now.
  bool add_granule(int i) {
    if (hipMemCreate(&h[i], gran, &prop_, 0) != hipSuccess) {
      (void)hipGetLastError();
      h[i] = nullptr;
      return false;
    }
    // a step that fails undoes the ones before it: the broker keeps running without this granule
    // (a transient shortage of address space or of the runtime's bookkeeping), grow() retries later
    hipMemAccessDesc d = rw();
    bool mapped = false;
    hipError_t e = hipMemExportToShareableHandle(&fds[i], h[i], hipMemHandleTypePosixFileDescriptor, 0);
    if (e == hipSuccess) e = hipMemAddressReserve(reinterpret_cast<void**>(&va[i]), gran, 0, nullptr, 0);
    if (e == hipSuccess) e = hipMemMap(va[i], gran, 0, h[i], 0), mapped = e == hipSuccess;
    if (e == hipSuccess) e = hipMemSetAccess(va[i], gran, &d, 1);
    if (e != hipSuccess) {
      std::fprintf(stderr, "gpushare-hbm-broker: granule %d not added: %s\n", i, hipGetErrorString(e));
      (void)hipGetLastError();
      if (mapped) (void)hipMemUnmap(va[i], gran);
      if (va[i]) (void)hipMemAddressFree(va[i], gran), va[i] = nullptr;
      (void)hipMemRelease(h[i]);
      h[i] = nullptr;
      if (fds[i] >= 0) close(fds[i]), fds[i] = -1;
      return false;
    }
    present[i] = 1;
    return true;
  }

  // granule i back to the driver (it is free: nobody holds it, it is not being scrubbed). The
  // driver wipes it when the last reference to its memory is gone.
  void destroy_granule(int i) {
    if (!present[i]) return;
    hipError_t e = hipMemUnmap(va[i], gran);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      std::fprintf(stderr, "gpushare-hbm-broker: unmap of granule %d: %s (kept out of the free list)\n", i,
                   hipGetErrorString(e));
      ++lost;
      return;
    }
    (void)hipMemRelease(h[i]);
    h[i] = nullptr;
    (void)hipMemAddressFree(va[i], gran);
    va[i] = nullptr;
    close(fds[i]);
    fds[i] = -1;
    base_refs[i] = -1;
    present[i] = 0;
    --count;
    ++given_back;
  }

  // whether the kernel reports a dma-buf's references in fdinfo ("count:"), read on a throwaway
  // export of the smallest handle; -1 when even that cannot be had (the device is full)
  int probe_counted() {
    size_t mg = 0;
    if (hipMemGetAllocationGranularity(&mg, &prop_, hipMemAllocationGranularityMinimum) != hipSuccess || !mg) mg = 2u << 20;
    hipMemGenericAllocationHandle_t t = nullptr;
    if (hipMemCreate(&t, mg, &prop_, 0) != hipSuccess) {
      (void)hipGetLastError();
      return -1;
    }
    int fd = -1, r = -1;
    if (hipMemExportToShareableHandle(&fd, t, hipMemHandleTypePosixFileDescriptor, 0) == hipSuccess && fd >= 0) {
      r = fd_refs(fd) >= 0 ? 1 : 0;
      close(fd);
    } else {
      (void)hipGetLastError();
    }
    (void)hipMemRelease(t);
    return r;
  }

  // the release policy once the kernel's reference count is known (at start, or at the first
  // granule when the device was full then)
  void settle_policy(int i) {
    if (counted >= 0 || !present[i]) return;
    counted = base_refs[i] >= 0 ? 1 : 0;
    choose_policy();
  }

  void choose_policy() {
    if (counted < 0) return;
    if (policy_auto) {
      policy = counted ? kRefs : kExit;
    } else if (policy == kRefs && !counted) {
      std::fprintf(stderr, "gpushare-hbm-broker: --release-policy refs needs the dma-buf count in fdinfo, which this "
                           "kernel does not report\n");
      std::exit(2);
    }
  }

  // sized for `target` bytes; holds as much of it as the device has free now, or nothing with
  // --start-empty (the rest is taken later, by grow(): after a broker restart, pods of the
  // previous instance still hold theirs)
  void setup(size_t target_bytes, size_t free_now, bool start_empty) {
    CK(hipSetDevice(device));
    std::memset(&prop_, 0, sizeof prop_);
    prop_.type = hipMemAllocationTypePinned;
    prop_.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    prop_.location.type = hipMemLocationTypeDevice;
    prop_.location.id = device;
    size_t mg = 0;
    CK(hipMemGetAllocationGranularity(&mg, &prop_, hipMemAllocationGranularityMinimum));
    if (mg && gran % mg) gran = (gran + mg - 1) / mg * mg;
    count_max = int(target_bytes / gran);
    target = start_empty ? 0 : count_max;
    int n0 = std::min(target, int(free_now / gran));
    double t0 = now_s();
    h.assign(count_max, nullptr);
    fds.assign(count_max, -1);
    base_refs.assign(count_max, -1);
    present.assign(count_max, 0);
    va.assign(count_max, nullptr);
    for (int i = 0; i < n0; ++i) {
      if (!add_granule(i)) break;
      free_list.push_back(i);
      ++count;
    }
    CK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    load_scrub_kernel();
    std::vector<int> every;
    for (int i = 0; i < count; ++i) every.push_back(i);
    zero_granules(every);  // nobody sees what was there before
    CK(hipStreamSynchronize(stream));
    for (int i = 0; i < count; ++i) base_refs[i] = refs(i);
    counted = count ? (base_refs[0] >= 0 ? 1 : 0) : probe_counted();
    setup_s = now_s() - t0;
  }

  // take more of the device while the broker is short of its target: HBM that pods of a previous
  // broker instance held comes back to the driver when they exit (the dma-buf imports keep it
  // alive until then), and what was given back under pressure or by SIZE is taken again once the
  // driver has more than the reserve free. New granules are zeroed like released ones before
  // they are lent.
  void grow() {
    if (count >= target) return;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr <= reserve_bytes) return;
    int n = std::min(target - count, int((fr - reserve_bytes) / gran));
    if (n <= 0) return;
    std::vector<int> fresh;
    for (int i = 0; i < count_max && int(fresh.size()) < n; ++i) {
      if (present[i]) continue;
      if (!add_granule(i)) break;  // raced: try again later
      base_refs[i] = refs(i);
      settle_policy(i);
      fresh.push_back(i);
      ++count;
    }
    grown += fresh.size();
    if (!fresh.empty())
      std::fprintf(stderr, "gpushare-hbm-broker: grew by %zu granules to %d of %d\n", fresh.size(), count, target);
    scrub(fresh);
  }

  // granules no grant has a claim on: the broker's size less every grant (taken or not: a grant
  // not taken yet is a pod about to start) and what is borrowed beyond grants. Only these are
  // lent beyond a grant or given back under pressure, so a pod's owed granules always come.
  long uncommitted() const {
    long c = 0;
    for (auto& g : grants) c += g.second.granules;
    for (auto& kv : clients) c += kv.second.extra;
    return long(std::min(count, target)) - c;
  }

  // what EXTEND may lend now: free granules no grant claims, and none while a taker waits
  int lendable() const {
    for (auto& kv : clients)
      if (!kv.second.waiting.empty() || kv.second.owed > 0) return 0;
    long u = std::min<long>(uncommitted(), long(free_list.size()));
    return int(std::max(0L, u));
  }

  // free granules beyond the target go back to the driver
  void shrink_to_target() {
    while (count > target && !free_list.empty()) {
      int i = free_list.back();
      free_list.pop_back();
      destroy_granule(i);
    }
  }

  // the driver is short (pods' runtimes, their quota beyond the granules, processes without a
  // grant): free granules no grant claims go back to it until it has --low-water-gib free again.
  // grow() takes them back once the driver has more than the reserve free.
  void relieve_pressure(double t) {
    if (!low_water_bytes || free_list.empty() || t - last_pressure < 0.05) return;
    last_pressure = t;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr >= low_water_bytes) return;
    long k = long((low_water_bytes - fr + gran - 1) / gran);
    k = std::min<long>(k, std::min<long>(uncommitted(), long(free_list.size())));
    for (long j = 0; j < k; ++j) {
      int i = free_list.back();
      free_list.pop_back();
      destroy_granule(i);
      ++pressure_given;
    }
    if (k > 0)
      std::fprintf(stderr, "gpushare-hbm-broker: driver had %.2f GiB free: gave %ld granules back (%d held)\n",
                   double(fr) / double(1ull << 30), k, count);
  }

  // zero granules `s` (sorted) on the broker's stream: one launch per run of granules whose
  // ranges happen to be adjacent
  void zero_granules(const std::vector<int>& s) {
    char* p[8];
    size_t b[8];
    int n = 0;
    for (size_t i = 0; i < s.size();) {
      size_t j = i + 1;
      while (j < s.size() && va[size_t(s[j])] == va[size_t(s[j - 1])] + gran) ++j;
      p[n] = va[size_t(s[i])], b[n] = gran * (j - i), ++n;
      if (n == 8) zero_ranges(p, b, n), n = 0;
      i = j;
    }
    if (n) zero_ranges(p, b, n);
  }

  // zero the granules on the broker's stream; they are lent again from reap_scrubs(), in chunks
  // of scrub_chunk granules (an event each): a pod waiting for a retired pod's 128 granules gets
  // the first ones after ~2 ms of zeroing, not after all of it
  void scrub(const std::vector<int>& idx) {
    if (idx.empty()) return;
    double t_enq = now_s();
    std::vector<int> s(idx);
    std::sort(s.begin(), s.end());
    size_t step = scrub_chunk > 0 ? size_t(scrub_chunk) : s.size();
    for (size_t c = 0; c < s.size(); c += step) {
      size_t e = std::min(s.size(), c + step);
      zero_granules(std::vector<int>(s.begin() + long(c), s.begin() + long(e)));
      hipEvent_t ev;
      CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      CK(hipEventRecord(ev, stream));
      scrubbing.push_back({std::vector<int>(s.begin() + long(c), s.begin() + long(e)), ev, now_s()});
    }
    scrub_enqueue_s_max = std::max(scrub_enqueue_s_max, now_s() - t_enq);
  }

  // scrubs whose event has completed (they complete in stream order): granules back to the free list
  bool reap_scrubs() {
    bool any = false;
    while (!scrubbing.empty()) {
      hipError_t q = hipEventQuery(scrubbing.front().ev);
      if (q == hipErrorNotReady) break;
      if (q != hipSuccess) die("hipEventQuery(scrub)", q);
      Scrub& s = scrubbing.front();
      CK(hipEventDestroy(s.ev));
      scrub_s_last = now_s() - s.t0;
      scrub_s_total += scrub_s_last;
      scrubbed_bytes += gran * s.idx.size();
      for (int i : s.idx) {
        if (count > target) destroy_granule(i);  // SIZE asked for less while it was lent
        else free_list.push_back(i);
      }
      scrubbing.pop_front();
      any = true;
    }
    return any;
  }

  static void reply(int fd, const std::string& s) {
    // admin and pod replies are short (LIST aside) and the peer reads them at once; a peer that
    // does not read is dropped by its request deadline, never waited for
    size_t off = 0;
    while (off < s.size()) {
      ssize_t n = send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (n > 0) {
        off += size_t(n);
        continue;
      }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        pollfd p{fd, POLLOUT, 0};
        if (poll(&p, 1, 100) > 0) continue;
      }
      return;
    }
  }

  // the header ("FDS <k> <gran>[ <total> <limit>]", "MORE <k> <gran>" or "XFDS <k> <gran>"), then
  // the fds
  bool send_fds(int fd, const std::vector<int>& idx, const char* verb = "FDS", int total = -1, int limit = -1) {
    double t0 = now_s();
    bool ok = send_fds_inner(fd, idx, verb, total, limit);
    send_s_max = std::max(send_s_max, now_s() - t0);
    timespec w;
    clock_gettime(CLOCK_REALTIME, &w);
    last_send_at = double(w.tv_sec) + double(w.tv_nsec) * 1e-9;
    return ok;
  }

  bool send_fds_inner(int fd, const std::vector<int>& idx, const char* verb, int total, int limit) {
    char head[96];
    int n = total >= 0 ? std::snprintf(head, sizeof head, "%s %zu %zu %d %d\n", verb, idx.size(), gran, total,
                                       std::max(limit, total))
                       : std::snprintf(head, sizeof head, "%s %zu %zu\n", verb, idx.size(), gran);
    if (send(fd, head, n, MSG_NOSIGNAL) != n) return false;
    for (size_t i = 0; i < idx.size(); i += 200) {
      size_t k = std::min<size_t>(200, idx.size() - i);
      std::vector<int> batch(k);
      for (size_t j = 0; j < k; ++j) batch[j] = fds[idx[i + j]];
      char byte = 'f';
      iovec io{&byte, 1};
      std::vector<char> ctl(CMSG_SPACE(k * sizeof(int)));
      msghdr m{};
      m.msg_iov = &io;
      m.msg_iovlen = 1;
      m.msg_control = ctl.data();
      m.msg_controllen = ctl.size();
      cmsghdr* c = CMSG_FIRSTHDR(&m);
      c->cmsg_level = SOL_SOCKET;
      c->cmsg_type = SCM_RIGHTS;
      c->cmsg_len = CMSG_LEN(k * sizeof(int));
      std::memcpy(CMSG_DATA(c), batch.data(), k * sizeof(int));
      if (sendmsg(fd, &m, MSG_NOSIGNAL) != 1) return false;
    }
    return true;
  }

  std::vector<int> pop_free(int n) {
    std::vector<int> idx;
    for (int i = 0; i < n && !free_list.empty(); ++i) {
      idx.push_back(free_list.front());
      free_list.pop_front();
    }
    return idx;
  }

  // serve TAKEs in arrival order while granules last: granules still owed to streaming takers
  // and whole grants of plain TAKEs go to the earliest first, nobody overtakes a taker still
  // short of granules. A streaming TAKE is accepted at once whatever is free (its first batch may
  // be empty): it is then owed the rest, in the same order.
  void serve_waiting() {
    std::vector<std::pair<double, int>> order;
    for (auto& kv : clients)
      if (!kv.second.waiting.empty() || kv.second.owed > 0) order.push_back({kv.second.wait_since, kv.first});
    std::sort(order.begin(), order.end());
    bool blocked = false;  // an earlier taker is still short: later ones get nothing now
    std::vector<int> dead;
    for (auto& o : order) {
      auto ci = clients.find(o.second);
      if (ci == clients.end()) continue;
      Client& c = ci->second;
      if (c.owed > 0) {
        if (blocked) continue;
        std::vector<int> idx = pop_free(c.owed);
        if (!idx.empty()) {
          c.owed -= int(idx.size());
          c.held.insert(c.held.end(), idx.begin(), idx.end());
          ++more_msgs;
          if (!send_fds(c.fd, idx, "MORE")) dead.push_back(o.second);
        }
        if (c.owed > 0) blocked = true;
        continue;
      }
      auto g = grants.find(c.waiting);
      if (g == grants.end() || g->second.holder >= 0) continue;  // not granted yet, or held
      int n = g->second.granules;
      if (!c.stream && (blocked || size_t(n) > free_list.size())) {
        blocked = true;  // keep arrival order: no overtaking
        continue;
      }
      std::vector<int> idx = pop_free(blocked ? 0 : n);
      g->second.holder = o.second;
      if (policy == kExit && c.pidfd < 0) c.pidfd = pidfd_of(c.pid);  // while it is surely alive
      c.token = c.waiting;
      c.waiting.clear();
      c.held = idx;
      c.owed = n - int(idx.size());
      ++takes;
      take_wait_s_last = now_s() - c.wait_since;
      take_wait_s_max = std::max(take_wait_s_max, take_wait_s_last);
      streamed += c.stream;
      if (c.owed > 0) blocked = true;
      if (!send_fds(c.fd, idx, "FDS", c.stream ? n : -1, g->second.limit)) dead.push_back(o.second);
    }
    for (int fd : dead) drop(fd);
  }

  // other references to granule i's dma-buf: the kernel's fdinfo "count" is the file's
  // reference count without procfs's own; the broker's exported fd is one of them. -1 = unknown
  int refs(int i) const { return fds[i] < 0 ? -1 : fd_refs(fds[i]); }

  static int fd_refs(int fd) {
    char path[64];
    std::snprintf(path, sizeof path, "/proc/self/fdinfo/%d", fd);
    FILE* f = std::fopen(path, "r");
    if (!f) return -1;
    char line[256];
    int count = -1;
    while (std::fgets(line, sizeof line, f))
      if (std::sscanf(line, "count: %d", &count) == 1) break;
    std::fclose(f);
    return count < 0 ? -1 : count - 1;
  }

  // references beyond the broker's own: a tenant (or whoever it passed the fd to) still has it
  bool outside(int i) const {
    int r = refs(i);
    return r < 0 || size_t(i) >= base_refs.size() || base_refs[i] < 0 || r > base_refs[i];
  }

  // the granules a connection held; takes over `pfd` (the holder's pidfd, or -1)
  void release(const std::vector<int>& idx, int pfd) {
    double t0 = now_s();
    release_inner(idx, pfd);
    release_s_max = std::max(release_s_max, now_s() - t0);
  }

  void release_inner(const std::vector<int>& idx, int pfd) {
    if (policy == kTrust) {
      if (pfd >= 0) close(pfd);
      scrub(idx);
      return;
    }
    if (policy == kExit) {
      if (pfd < 0) {  // the holder cannot be followed: never lent again (fail closed)
        lost += idx.size();
        std::fprintf(stderr, "gpushare-hbm-broker: %zu granules of an untraceable holder are not lent again\n",
                     idx.size());
        return;
      }
      quarantined_total += idx.size();
      quarantine.push_back({idx, pfd, now_s()});
      return;
    }
    if (pfd >= 0) close(pfd);
    std::vector<int> clean, kept;
    for (int i : idx) (outside(i) ? kept : clean).push_back(i);
    scrub(clean);
    if (!kept.empty()) {
      quarantined_total += kept.size();
      quarantine.push_back({std::move(kept), -1, now_s()});
    }
  }

  void quarantine_done(const Held& g) {
    quarantine_s_last = now_s() - g.t0;
    quarantine_s_max = std::max(quarantine_s_max, quarantine_s_last);
  }

  size_t quarantined() const {
    size_t n = 0;
    for (auto& g : quarantine) n += g.idx.size();
    return n;
  }

  // quarantined granules whose holder is really gone: scrub (again) and lend. A release's
  // granules lose their references together (the tenant's process teardown), so while the
  // group's first one is still referenced the rest are not read.
  void sweep_quarantine() {
    std::vector<Held> keep;
    for (auto& g : quarantine) {
      if (g.pidfd >= 0) {
        if (!exited(g.pidfd)) {
          keep.push_back(std::move(g));
          continue;
        }
        close(g.pidfd);
        quarantine_done(g);
        scrub(g.idx);
        continue;
      }
      if (outside(g.idx.front())) {
        keep.push_back(std::move(g));
        continue;
      }
      std::vector<int> back, still;
      for (int i : g.idx) (outside(i) ? still : back).push_back(i);
      scrub(back);
      if (!still.empty()) keep.push_back({std::move(still), -1, g.t0});
      else quarantine_done(g);
    }
    quarantine.swap(keep);
  }

  void drop(int fd) {
    auto it = clients.find(fd);
    if (it == clients.end()) return;
    if (!it->second.held.empty()) {
      release(it->second.held, it->second.pidfd);
      ++releases;
    } else if (it->second.pidfd >= 0) {
      close(it->second.pidfd);
    }
    auto g = it->second.token.empty() ? grants.end() : grants.find(it->second.token);
    if (g != grants.end() && g->second.holder == fd) {
      g->second.holder = -1;
      g->second.at = now_s();
    }
    close(fd);
    clients.erase(it);
  }

  int held_refs_max() const {  // references beyond the baseline, over the granules lent out
    int m = -1;
    for (auto& kv : clients)
      for (int i : kv.second.held) m = std::max(m, refs(i) - (size_t(i) < base_refs.size() ? base_refs[i] : 0));
    return m;
  }

  const char* policy_name() const { return policy == kRefs ? "refs" : policy == kExit ? "exit" : "trust"; }

  std::string stat() const {
    size_t held = 0, waiting = 0, scrub_n = 0, owed = 0, extra = 0;
    for (auto& kv : clients) {
      held += kv.second.held.size();
      waiting += !kv.second.waiting.empty();
      owed += size_t(kv.second.owed);
      extra += size_t(kv.second.extra);
    }
    for (auto& s : scrubbing) scrub_n += s.idx.size();
    char b[4096];
    int n = std::snprintf(b, sizeof b,
                  "{\"boot\": \"%s\", \"device\": %d, \"granule_bytes\": %zu, \"granules\": %d, \"granules_max\": %d, "
                  "\"target\": %d, \"given_back\": %llu, \"pressure_given\": %llu, \"low_water_bytes\": %zu, "
                  "\"extra\": %zu, \"extends\": %llu, \"extended\": %llu, \"uncommitted\": %ld, \"ends\": %llu, "
                  "\"grown\": %llu, \"free\": %zu, "
                  "\"held\": %zu, \"owed\": %zu, \"streamed\": %llu, \"more_msgs\": %llu, \"scrubbing\": %zu, \"waiting\": %zu, \"grants\": %zu, \"takes\": %llu, "
                  "\"releases\": %llu, \"refused\": %llu, \"revokes\": %llu, \"revoked\": %zu, \"timeouts\": %llu, "
                  "\"expired\": %llu, \"busy\": %llu, \"idle_dropped\": %llu, \"peer_refused\": %llu, "
                  "\"clients\": %zu, \"quarantined\": %zu, \"quarantined_total\": %llu, \"lost\": %llu, "
                  "\"scrub_kernel\": \"%s\", \"scrub_dispatches\": %llu, \"release_policy\": \"%s\", \"quarantine_ms_last\": %.1f, \"quarantine_ms_max\": %.1f, \"held_refs_max\": %d, \"base_refs\": %d, \"scrubbed_bytes\": %llu, "
                  "\"scrub_ms_total\": %.3f, \"scrub_ms_last\": %.3f, \"setup_ms\": %.1f, \"loop_ms_max\": %.3f, "
                  "\"release_ms_max\": %.3f, \"scrub_enqueue_ms_max\": %.3f, \"take_wait_ms_last\": %.3f, "
                  "\"take_wait_ms_max\": %.3f, \"send_ms_max\": %.3f, \"last_send_at\": %.6f}\n",
                  boot.c_str(), device, gran, count, count_max, target, given_back, pressure_given, low_water_bytes,
                  extra, extends, extended, uncommitted(), ends, grown, free_list.size(), held, owed, streamed, more_msgs, scrub_n, waiting, grants.size(), takes,
                  releases, refused, revokes, revoked.size(), timeouts, expired, busy, idle_dropped, peer_refused,
                  clients.size(), quarantined(), quarantined_total, lost,
                  scrub_n_fn ? "gs_scrub_n" : scrub_fn ? "gs_scrub" : "memset", scrub_dispatches, policy_name(),
                  quarantine_s_last * 1e3,
                  quarantine_s_max * 1e3, held_refs_max(),
                  base_refs.empty() ? -1 : base_refs[0], scrubbed_bytes, scrub_s_total * 1e3, scrub_s_last * 1e3,
                  setup_s * 1e3, loop_s_max * 1e3, release_s_max * 1e3, scrub_enqueue_s_max * 1e3,
                  take_wait_s_last * 1e3, take_wait_s_max * 1e3, send_s_max * 1e3, last_send_at);
    return n > 0 && size_t(n) < sizeof b ? std::string(b) : std::string("{}\n");
  }

  std::string list() const {
    std::string s = "{\"boot\": \"" + boot + "\", \"grants\": {";
    bool first = true;
    for (auto& kv : grants) {
      s += (first ? "\"" : ", \"") + kv.first + "\": " + std::to_string(kv.second.granules);
      first = false;
    }
    return s + "}}\n";
  }

  void remember_revoked(const std::string& t) {
    if (revoked.insert(t).second) {
      revoked_order.push_back(t);
      while (revoked_order.size() > 65536) {
        revoked.erase(revoked_order.front());
        revoked_order.pop_front();
      }
    }
  }

  // the words of a request line (single spaces; anything else is not a request)
  static std::vector<std::string> words(const std::string& line) {
    std::vector<std::string> w;
    size_t i = 0;
    while (i <= line.size()) {
      size_t j = line.find(' ', i);
      if (j == std::string::npos) j = line.size();
      w.push_back(line.substr(i, j - i));
      i = j + 1;
    }
    return w;
  }

  // decimal digits only, no overflow
  static bool u64(const std::string& s, unsigned long long* v) {
    if (s.empty() || s.size() > 20) return false;
    unsigned long long x = 0;
    for (char ch : s) {
      if (ch < '0' || ch > '9') return false;
      unsigned d = unsigned(ch - '0');
      if (x > (~0ull - d) / 10) return false;
      x = x * 10 + d;
    }
    *v = x;
    return true;
  }

  // "TAKE <token>" or "TAKE <token> STREAM"
  static bool take_line(const std::string& line, char* tok, bool* stream) {
    char opt[16] = {0};
    char extra = 0;
    int k = std::sscanf(line.c_str(), "TAKE %128s %15s %c", tok, opt, &extra);
    if (!valid_token(tok)) return false;
    if (k == 1) {
      *stream = false;
      return true;
    }
    if (k == 2 && std::strcmp(opt, "STREAM") == 0) {
      *stream = true;
      return true;
    }
    return false;
  }

  // "EXTEND <k>": granules beyond the grant for a holder that is owed nothing, up to its limit,
  // from granules no grant claims; "XFDS 0" when there are none (the pod uses the driver)
  void extend(int fd, Client& c, unsigned long long k) {
    auto g = c.token.empty() ? grants.end() : grants.find(c.token);
    int j = 0;
    if (g != grants.end() && g->second.holder == fd) {
      long room = long(g->second.limit) - long(c.held.size());
      j = int(std::max(0L, std::min<long>({long(std::min<unsigned long long>(k, 1u << 20)), room, long(lendable())})));
    }
    std::vector<int> idx = pop_free(j);
    c.held.insert(c.held.end(), idx.begin(), idx.end());
    c.extra += int(idx.size());
    ++extends;
    extended += idx.size();
    if (!send_fds(fd, idx, "XFDS")) drop(fd);
  }

  int avail(int fd, const Client& c) const {
    auto g = c.token.empty() ? grants.end() : grants.find(c.token);
    if (g == grants.end() || g->second.holder != fd || c.owed > 0) return 0;
    return int(std::max(0L, std::min<long>(long(g->second.limit) - long(c.held.size()), long(lendable()))));
  }

  void on_line(int fd, const std::string& line) {
    Client& c = clients[fd];
    c.asked = true;
    char tok[129] = {0};
    std::vector<std::string> w = words(line);
    unsigned long long bytes = 0, limit = 0, k = 0;
    std::string tk = w.size() > 1 ? w[1] : std::string();
    bool tok_ok = tk.size() <= 128 && valid_token(tk.c_str());
    if (tok_ok) std::memcpy(tok, tk.c_str(), tk.size() + 1);
    if (c.admin && w[0] == "GRANT" && (w.size() == 3 || w.size() == 4) && tok_ok && u64(w[2], &bytes) &&
        (w.size() == 3 || u64(w[3], &limit))) {
      // in granules, without overflow: bytes beyond the broker's size are refused before rounding
      // (a broker still growing honours a grant up to its full size as its granules arrive)
      unsigned long long cap = (unsigned long long)count_max * (unsigned long long)gran;
      if (bytes == 0 || bytes > cap) {
        ++refused;
        reply(fd, "ERR size\n");
        return;
      }
      int n = int(bytes / gran + (bytes % gran ? 1 : 0));
      int lim = int(std::min<unsigned long long>(std::max(limit, bytes), cap) / gran);  // whole granules of the quota
      auto& gr = grants[tok];  // a repeated grant (a re-prepared answer, a re-grant) refreshes it
      gr.granules = n;
      gr.limit = std::max(lim, n);
      gr.at = now_s();
      if (revoked.erase(tok)) revoked_order.erase(std::find(revoked_order.begin(), revoked_order.end(), std::string(tok)));
      reply(fd, "OK " + std::to_string(n) + "\n");
      serve_waiting();
    } else if (c.admin && w[0] == "SIZE" && w.size() == 2 && (w[1] == "max" || u64(w[1], &k))) {
      target = w[1] == "max" ? count_max : int(std::min<unsigned long long>(k, (unsigned long long)count_max));
      shrink_to_target();
      grow();
      reply(fd, "OK " + std::to_string(count) + " " + std::to_string(target) + "\n");
    } else if (c.admin && w[0] == "REVOKE" && w.size() == 2 && tok_ok) {
      std::string t(tok);
      int held = 0;
      auto g = grants.find(t);
      if (g != grants.end()) {
        if (g->second.holder >= 0) {
          auto h = clients.find(g->second.holder);
          if (h != clients.end()) {
            h->second.token.clear();  // its end returns the granules, the grant is gone already
            h->second.owed = 0;       // and it is lent no more of them: it is told so
            held = int(h->second.held.size());
            reply(h->first, "END\n");
            ++ends;
          }
        }
        grants.erase(g);
      }
      remember_revoked(t);
      ++revokes;
      std::vector<int> waiters;
      for (auto& kv : clients)
        if (kv.second.waiting == t) waiters.push_back(kv.first);
      for (int w : waiters) {
        reply(w, "ERR revoked\n");
        drop(w);
      }
      reply(fd, "OK " + std::to_string(held) + "\n");
    } else if (c.admin && line == "LIST") {
      reply(fd, list());
    } else if (c.admin && line == "STAT") {
      reply(fd, stat());
    } else if (!c.admin && w[0] == "EXTEND" && w.size() == 2 && u64(w[1], &k) && k > 0 && !c.token.empty() &&
               c.owed == 0 && c.waiting.empty()) {
      extend(fd, c, k);
    } else if (!c.admin && line == "AVAIL" && !c.token.empty() && c.waiting.empty()) {
      reply(fd, "AVAIL " + std::to_string(avail(fd, c)) + "\n");
    } else if (!c.admin && (w[0] == "EXTEND" || line == "AVAIL") && c.waiting.empty() && !c.held.empty()) {
      // a holder whose grant was revoked: nothing more
      reply(fd, w[0] == "EXTEND" ? "XFDS 0 " + std::to_string(gran) + "\n" : std::string("AVAIL 0\n"));
    } else if (!c.admin && c.held.empty() && c.waiting.empty() && c.token.empty() && take_line(line, tok, &c.stream)) {
      if (revoked.count(tok)) {
        ++refused;
        reply(fd, "ERR revoked\n");
        drop(fd);
        return;
      }
      c.waiting = tok;
      c.wait_since = now_s();
      serve_waiting();
    } else {
      ++refused;
      reply(fd, "ERR request\n");
    }
  }

  // one connection from a listener; false when there is none left to accept
  bool accept_one(int ls, bool admin) {
    int c = accept4(ls, nullptr, nullptr, SOCK_CLOEXEC | SOCK_NONBLOCK);
    if (c < 0) return false;
    ucred cr{};
    socklen_t cl = sizeof cr;
    bool have_cred = getsockopt(c, SOL_SOCKET, SO_PEERCRED, &cr, &cl) == 0;
    if (admin && (!have_cred || (cr.uid != 0 && cr.uid != geteuid()))) {
      ++peer_refused;  // the socket's mode already says this; the peer's credentials say it again
      reply(c, "ERR peer\n");
      close(c);
      return true;
    }
    size_t same = 0;
    if (!admin && have_cred && cr.pid > 0)
      for (auto& kv : clients) same += !kv.second.admin && kv.second.pid == cr.pid;
    if (clients.size() >= max_clients || same >= max_per_peer) {
      ++busy;
      reply(c, "ERR busy\n");
      close(c);
      return true;
    }
    Client& n = clients[c];
    n.fd = c;
    n.admin = admin;
    n.since = now_s();
    n.pid = have_cred ? cr.pid : 0;
    n.uid = have_cred ? cr.uid : 0;
    return true;
  }
};

}  // namespace

int main(int argc, char** argv) {
  std::string sock, admin, pci, policy = "auto";
  Broker b;
  double gib = 0, reserve_gib = 16, low_water_gib = -1;
  size_t gran_mib = 1024;
  bool start_empty = false;
  for (int i = 1; i < argc; i += 2) {
    std::string k = argv[i];
    if (k == "--start-empty") {
      start_empty = true;
      --i;
      continue;
    }
    if (i + 1 >= argc) {
      std::fprintf(stderr, "gpushare-hbm-broker: %s needs a value\n", k.c_str());
      return 2;
    }
    const char* v = argv[i + 1];
    if (k == "--socket") sock = v;
    else if (k == "--admin-socket") admin = v;
    else if (k == "--device") b.device = std::atoi(v);
    else if (k == "--pci-bus-id") pci = v;  // the GPU by PCI address (HIP and SMI orders differ)
    else if (k == "--gib") gib = std::atof(v);
    else if (k == "--reserve-gib") reserve_gib = std::atof(v);
    else if (k == "--granule-mib") gran_mib = std::strtoull(v, nullptr, 10);
    else if (k == "--wait-s") b.wait_s = std::atof(v);
    else if (k == "--ungranted-wait-s") b.ungranted_wait_s = std::atof(v);
    else if (k == "--grant-ttl-s") b.grant_ttl_s = std::atof(v);
    else if (k == "--max-clients") b.max_clients = std::strtoull(v, nullptr, 10);
    else if (k == "--max-per-peer") b.max_per_peer = std::strtoull(v, nullptr, 10);
    else if (k == "--request-timeout-s") b.request_timeout_s = std::atof(v);
    else if (k == "--release-policy") policy = v;
    else if (k == "--scrub-chunk") b.scrub_chunk = std::atoi(v);
    else if (k == "--scrub-kernel") b.scrub_path = v;
    else if (k == "--low-water-gib") low_water_gib = std::atof(v);
    else {
      std::fprintf(stderr, "gpushare-hbm-broker: unknown flag %s\n", k.c_str());
      return 2;
    }
  }
  if (sock.empty() || (policy != "auto" && policy != "refs" && policy != "exit" && policy != "trust")) {
    std::fprintf(stderr, "usage: gpushare-hbm-broker --socket PATH [--admin-socket PATH] [--device N | --pci-bus-id BDF] "
                         "[--gib N | --reserve-gib N] [--granule-mib 1024] [--wait-s 30] [--ungranted-wait-s 10] "
                         "[--release-policy auto|refs|exit|trust] [--start-empty] [--low-water-gib N]\n");
    return 2;
  }
  if (admin.empty()) admin = sock + ".admin";
  if (b.scrub_path.empty()) {  // default: next to this executable
    char self[4096];
    ssize_t n = readlink("/proc/self/exe", self, sizeof self - 1);
    if (n > 0) {
      self[n] = 0;
      std::string dir(self);
      b.scrub_path = dir.substr(0, dir.rfind('/') + 1) + "gpushare-hbm-scrub.co";
    }
  }
  b.gran = gran_mib << 20;
  if (!pci.empty()) CK(hipDeviceGetByPCIBusId(&b.device, pci.c_str()));
  CK(hipSetDevice(b.device));
  size_t fr = 0, tot = 0;
  CK(hipMemGetInfo(&fr, &tot));
  b.reserve_bytes = size_t(reserve_gib * double(1ull << 30));
  // sized for the device (or --gib); what is not free yet is taken as it comes back (grow): pods
  // of a previous broker instance, or memory amdgpu is still wiping after another process
  size_t target = gib > 0 ? size_t(gib * double(1ull << 30)) : (tot > b.reserve_bytes ? tot - b.reserve_bytes : 0);
  if (gib > 0) b.reserve_bytes = size_t(2) << 30;  // --gib: leave the driver a small margin while growing
  size_t free_now = fr > b.reserve_bytes ? fr - b.reserve_bytes : 0;
  b.low_water_bytes = size_t((low_water_gib >= 0 ? low_water_gib : double(b.reserve_bytes) / double(1ull << 30) / 2) *
                             double(1ull << 30));
  b.setup(target, std::min(target, free_now), start_empty);
  // the release policy: auto = refs where the kernel counts a dma-buf's references. Known from the
  // first granule, or a throwaway export when there is none; on a full device, at the first
  // granule grown (nothing can be lent before it)
  b.policy_auto = policy == "auto";
  b.policy = policy == "refs" ? kRefs : policy == "exit" ? kExit : policy == "trust" ? kTrust : kRefs;
  b.choose_policy();
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  signal(SIGPIPE, SIG_IGN);
  int pod_ls = listen_unix(sock, 0666);
  int adm_ls = listen_unix(admin, 0600);
  std::printf("{\"ready\": true, \"boot\": \"%s\", \"socket\": \"%s\", \"admin_socket\": \"%s\", \"granules\": %d, "
              "\"granule_bytes\": %zu, \"release_policy\": \"%s\", \"scrub_kernel\": \"%s\", \"setup_ms\": %.1f}\n",
              b.boot.c_str(), sock.c_str(), admin.c_str(), b.count, b.gran, b.policy_name(),
              b.scrub_fn ? "gs_scrub" : "memset", b.setup_s * 1e3);
  std::fflush(stdout);

  std::vector<pollfd> pf;
  double last_grow = now_s();
  while (!g_stop) {
    pf.assign({{pod_ls, POLLIN, 0}, {adm_ls, POLLIN, 0}});
    for (auto& kv : b.clients) pf.push_back({kv.first, POLLIN, 0});
    // scrubs complete on the GPU in a few ms, and a retired tenant's references drop when the
    // kernel finishes tearing its process down: look often while granules wait for either
    int timeout = !b.scrubbing.empty() ? 1 : !b.quarantine.empty() ? 3 : 100;
    int r = poll(pf.data(), pf.size(), timeout);
    if (r < 0 && errno != EINTR) break;
    double t_pass = now_s();
    for (int k = 0; k < 2 && r > 0; ++k)
      if (pf[k].revents & POLLIN)
        for (int j = 0; j < 64 && b.accept_one(pf[k].fd, k == 1); ++j) {
        }  // drain the backlog, bounded per pass
    for (size_t k = 2; k < pf.size() && r > 0; ++k) {
      if (!pf[k].revents) continue;
      int fd = pf[k].fd;
      if (!b.clients.count(fd)) continue;
      char buf[512];
      ssize_t n = recv(fd, buf, sizeof buf, 0);
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) continue;
      if (n <= 0) {  // the pod is gone (or the admin hung up): scrub and return its granules
        b.drop(fd);
        b.serve_waiting();
        continue;
      }
      Client& c = b.clients[fd];
      c.in.append(buf, size_t(n));
      if (c.in.size() > 4096) {
        b.drop(fd);
        continue;
      }
      size_t nl;
      while (b.clients.count(fd) && (nl = b.clients[fd].in.find('\n')) != std::string::npos) {
        std::string line = b.clients[fd].in.substr(0, nl);
        b.clients[fd].in.erase(0, nl + 1);
        b.on_line(fd, line);
      }
    }
    double t = now_s();
    std::vector<int> late, idle, ended;
    for (auto& kv : b.clients) {
      const Client& c = kv.second;
      if (c.owed > 0 && t - c.wait_since > b.wait_s) {
        ended.push_back(kv.first);   // owed granules that did not come in time: cancelled
      } else if (!c.waiting.empty()) {
        // TAKEs that waited too long are refused (their grant stays for a retry); a TAKE with no
        // grant at all gets a shorter deadline than one waiting for a retiring pod's granules
        bool granted = b.grants.count(c.waiting) > 0;
        if (t - c.wait_since > (granted ? b.wait_s : b.ungranted_wait_s)) late.push_back(kv.first);
      } else if (!c.asked && t - c.since > b.request_timeout_s) {
        idle.push_back(kv.first);  // connected, never asked: junk or a stuck peer
      }
    }
    for (int fd : late) {
      ++b.timeouts;
      bool granted = b.grants.count(b.clients[fd].waiting) > 0;
      Broker::reply(fd, granted ? "ERR timeout\n" : "ERR nogrant\n");
      b.drop(fd);
    }
    for (int fd : idle) {
      ++b.idle_dropped;
      b.drop(fd);
    }
    for (int fd : ended) {
      // the shim takes any line but MORE as the end of its stream: its grant (and its ledger
      // charge) shrinks to what it has, and it allocates the rest from the driver. A taker still
      // owed granules no longer holds up the ones behind it.
      ++b.ends;
      b.clients[fd].owed = 0;
      Broker::reply(fd, "END\n");
    }
    bool back = b.reap_scrubs();
    if (!b.quarantine.empty()) b.sweep_quarantine();
    if (b.count < b.target && t - last_grow > 1.0) {
      last_grow = t;
      b.grow();
    }
    b.relieve_pressure(t);
    if (back || !late.empty() || !ended.empty()) b.serve_waiting();
    b.loop_s_max = std::max(b.loop_s_max, now_s() - t_pass);
    // with a TTL, grants of pods that never started (deleted before admission) do not pile up;
    // without one (the default) the plugin's revocations do that
    if (b.grant_ttl_s > 0)
      for (auto it = b.grants.begin(); it != b.grants.end();) {
        if (it->second.holder < 0 && t - it->second.at > b.grant_ttl_s) {
          it = b.grants.erase(it);
          ++b.expired;
        } else {
          ++it;
        }
      }
  }
  for (auto it = b.clients.begin(); it != b.clients.end();) close((it++)->first);
  if (!b.scrubbing.empty()) (void)hipStreamSynchronize(b.stream);
  unlink(sock.c_str());
  unlink(admin.c_str());
  return 0;
}
