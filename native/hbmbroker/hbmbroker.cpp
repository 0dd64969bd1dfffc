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
// (the device plugin's Allocate, or the bench acting for it) on an admin socket that only root
// can open, and a pod takes its grant with its token (again after a container restart).
//
// Protocol: one text line per connection's request.
//   admin socket  <sock>.admin (0600):  "GRANT <token> <bytes>\n"  -> "OK <granules>\n" | "ERR ...\n"
//                                       "STAT\n"                   -> one JSON line
//   pod socket    <sock>       (0666):  "TAKE <token>\n"           -> "FDS <n> <granule bytes>\n",
//                                        then n fds (batches of <= 200, one byte each); the
//                                        connection stays open: its end (close, exit, crash)
//                                        returns the granules, which are scrubbed first.
// A TAKE whose grant has not arrived yet, or whose granules are still held by a retiring pod,
// waits (up to --wait-s) instead of failing: the pod's runtime may start before the retired pod
// is gone, as it does on a node.
//
//   gpushare-hbm-broker --socket /run/gpushare/hbm0.sock [--device 0 | --pci-bus-id 0000:05:00.0]
//                       [--gib N | --reserve-gib R]
//                       [--granule-mib 1024] [--wait-s 30] [--grant-ttl-s 600]
#include <hip/hip_runtime.h>

#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
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
  int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  if (path.size() >= sizeof a.sun_path) {
    std::fprintf(stderr, "gpushare-hbm-broker: socket path too long: %s\n", path.c_str());
    std::exit(2);
  }
  std::memcpy(a.sun_path, path.c_str(), path.size() + 1);
  unlink(path.c_str());
  if (bind(s, reinterpret_cast<sockaddr*>(&a), sizeof a) || listen(s, 64)) {
    std::perror(path.c_str());
    std::exit(2);
  }
  chmod(path.c_str(), mode);
  return s;
}

struct Client {
  int fd = -1;
  bool admin = false;
  std::string in;
  // a pod: the granules it holds (indices), or the token it waits for
  std::vector<int> held;
  std::string token;    // the grant it holds
  std::string waiting;  // token of a TAKE not yet served
  double wait_since = 0;
};

struct Broker {
  int device = 0;
  size_t gran = 1ull << 30;
  int count = 0;
  double wait_s = 30.0;
  std::vector<hipMemGenericAllocationHandle_t> h;
  std::vector<int> fds;
  char* base = nullptr;  // every granule mapped here, for the scrub
  hipStream_t stream = nullptr;
  std::deque<int> free_list;
  // granules whose dma-buf something besides the broker still refers to (a tenant kept an fd, or
  // passed it on): not lent again until that reference is gone, then scrubbed again
  std::vector<std::vector<int>> quarantine;  // by release: one tenant's granules go together
  unsigned long long quarantined_total = 0;
  std::vector<int> base_refs;  // each granule's references with no tenant (the broker's own export)
  // A grant belongs to the pod, not to one process: a TAKE holds it while its connection lives,
  // and a restarted container (same env, same token) takes it again once the old process's
  // granules are back. It expires grant_ttl_s after it was granted or last released.
  struct Grant {
    int granules;
    double at;
    int holder = -1;  // fd of the connection holding it
  };
  std::map<std::string, Grant> grants;
  double grant_ttl_s = 600.0;
  unsigned long long expired = 0;
  std::map<int, Client> clients;
  // stats
  unsigned long long takes = 0, releases = 0, refused = 0, timeouts = 0;
  double scrub_s_total = 0, scrub_s_last = 0, setup_s = 0;
  unsigned long long scrubbed_bytes = 0;

  void setup(size_t total) {
    CK(hipSetDevice(device));
    hipMemAllocationProp p;
    std::memset(&p, 0, sizeof p);
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = device;
    size_t mg = 0;
    CK(hipMemGetAllocationGranularity(&mg, &p, hipMemAllocationGranularityMinimum));
    if (mg && gran % mg) gran = (gran + mg - 1) / mg * mg;
    count = int(total / gran);
    double t0 = now_s();
    h.resize(count);
    fds.resize(count);
    CK(hipMemAddressReserve(reinterpret_cast<void**>(&base), gran * count, 0, nullptr, 0));
    for (int i = 0; i < count; ++i) {
      CK(hipMemCreate(&h[i], gran, &p, 0));
      CK(hipMemExportToShareableHandle(&fds[i], h[i], hipMemHandleTypePosixFileDescriptor, 0));
      CK(hipMemMap(base + size_t(i) * gran, gran, 0, h[i], 0));
      free_list.push_back(i);
    }
    hipMemAccessDesc d;
    std::memset(&d, 0, sizeof d);
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = device;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(base, gran * count, &d, 1));
    CK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    CK(hipMemsetAsync(base, 0, gran * count, stream));  // nobody sees what was there before
    CK(hipStreamSynchronize(stream));
    base_refs.resize(count);
    for (int i = 0; i < count; ++i) base_refs[i] = refs(i);
    setup_s = now_s() - t0;
  }

  void scrub(const std::vector<int>& idx) {
    if (idx.empty()) return;
    double t0 = now_s();
    std::vector<int> s(idx);
    std::sort(s.begin(), s.end());
    for (size_t i = 0; i < s.size();) {  // one memset per run of adjacent granules
      size_t j = i + 1;
      while (j < s.size() && s[j] == s[j - 1] + 1) ++j;
      CK(hipMemsetAsync(base + size_t(s[i]) * gran, 0, gran * (j - i), stream));
      i = j;
    }
    CK(hipStreamSynchronize(stream));
    scrub_s_last = now_s() - t0;
    scrub_s_total += scrub_s_last;
    scrubbed_bytes += gran * idx.size();
  }

  static void reply(int fd, const std::string& s) { (void)!send(fd, s.data(), s.size(), MSG_NOSIGNAL); }

  bool send_fds(int fd, const std::vector<int>& idx) {
    char head[64];
    int n = std::snprintf(head, sizeof head, "FDS %zu %zu\n", idx.size(), gran);
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

  // serve waiting TAKEs in arrival order while granules last
  void serve_waiting() {
    std::vector<std::pair<double, int>> order;
    for (auto& kv : clients)
      if (!kv.second.waiting.empty()) order.push_back({kv.second.wait_since, kv.first});
    std::sort(order.begin(), order.end());
    for (auto& o : order) {
      Client& c = clients[o.second];
      auto g = grants.find(c.waiting);
      if (g == grants.end() || g->second.holder >= 0) continue;  // not granted yet, or held
      if (size_t(g->second.granules) > free_list.size()) break;  // keep arrival order: no overtaking
      std::vector<int> idx;
      for (int i = 0; i < g->second.granules; ++i) {
        idx.push_back(free_list.front());
        free_list.pop_front();
      }
      g->second.holder = o.second;
      c.token = c.waiting;
      c.waiting.clear();
      c.held = idx;
      ++takes;
      if (!send_fds(c.fd, idx)) drop(o.second);
    }
  }

  // other references to granule i's dma-buf: the kernel's fdinfo "count" is the file's
  // reference count without procfs's own; the broker's exported fd is one of them. -1 = unknown
  // (no such field: then the release is trusted, as before)
  int refs(int i) const {
    char path[64];
    std::snprintf(path, sizeof path, "/proc/self/fdinfo/%d", fds[i]);
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
    return r >= 0 && size_t(i) < base_refs.size() && base_refs[i] >= 0 && r > base_refs[i];
  }

  void release(const std::vector<int>& idx) {
    std::vector<int> clean, held;
    for (int i : idx) (outside(i) ? held : clean).push_back(i);
    scrub(clean);
    for (int i : clean) free_list.push_back(i);
    if (!held.empty()) {
      quarantined_total += held.size();
      quarantine.push_back(std::move(held));
    }
  }

  size_t quarantined() const {
    size_t n = 0;
    for (auto& g : quarantine) n += g.size();
    return n;
  }

  // quarantined granules whose last outside reference is gone: scrub (again) and lend. A
  // release's granules lose their references together (the tenant's process teardown), so
  // while the group's first one is still referenced the rest are not read.
  bool sweep_quarantine() {
    bool any = false;
    std::vector<std::vector<int>> keep;
    for (auto& g : quarantine) {
      if (outside(g.front())) {
        keep.push_back(std::move(g));
        continue;
      }
      std::vector<int> back, still;
      for (int i : g) (outside(i) ? still : back).push_back(i);
      scrub(back);
      for (int i : back) free_list.push_back(i);
      any = any || !back.empty();
      if (!still.empty()) keep.push_back(std::move(still));
    }
    quarantine.swap(keep);
    return any;
  }

  void drop(int fd) {
    auto it = clients.find(fd);
    if (it == clients.end()) return;
    if (!it->second.held.empty()) {
      release(it->second.held);
      ++releases;
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

  std::string stat() const {
    size_t held = 0, waiting = 0;
    for (auto& kv : clients) {
      held += kv.second.held.size();
      waiting += !kv.second.waiting.empty();
    }
    char b[1024];
    std::snprintf(b, sizeof b,
                  "{\"device\": %d, \"granule_bytes\": %zu, \"granules\": %d, \"free\": %zu, \"held\": %zu, "
                  "\"waiting\": %zu, \"grants\": %zu, \"takes\": %llu, \"releases\": %llu, \"refused\": %llu, "
                  "\"timeouts\": %llu, \"expired\": %llu, \"quarantined\": %zu, \"quarantined_total\": %llu, "
                  "\"held_refs_max\": %d, \"base_refs\": %d, \"scrubbed_bytes\": %llu, \"scrub_ms_total\": %.3f, \"scrub_ms_last\": %.3f, "
                  "\"setup_ms\": %.1f}\n",
                  device, gran, count, free_list.size(), held, waiting, grants.size(), takes, releases, refused,
                  timeouts, expired, quarantined(), quarantined_total, held_refs_max(), base_refs.empty() ? -1 : base_refs[0], scrubbed_bytes, scrub_s_total * 1e3, scrub_s_last * 1e3, setup_s * 1e3);
    return b;
  }

  void on_line(int fd, const std::string& line) {
    Client& c = clients[fd];
    char tok[129] = {0};
    unsigned long long bytes = 0;
    if (c.admin && std::sscanf(line.c_str(), "GRANT %128s %llu", tok, &bytes) == 2) {
      int n = int((bytes + gran - 1) / gran);
      if (n <= 0 || n > count) {
        ++refused;
        reply(fd, "ERR size\n");
        return;
      }
      auto& gr = grants[tok];  // a repeated grant (a re-prepared answer) refreshes it
      gr.granules = n;
      gr.at = now_s();
      reply(fd, "OK " + std::to_string(n) + "\n");
      serve_waiting();
    } else if (c.admin && line == "STAT") {
      reply(fd, stat());
    } else if (!c.admin && c.held.empty() && c.waiting.empty() && std::sscanf(line.c_str(), "TAKE %128s", tok) == 1) {
      c.waiting = tok;
      c.wait_since = now_s();
      serve_waiting();
    } else {
      ++refused;
      reply(fd, "ERR request\n");
    }
  }
};

}  // namespace

int main(int argc, char** argv) {
  std::string sock, pci;
  Broker b;
  double gib = 0, reserve_gib = 16;
  size_t gran_mib = 1024;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i];
    const char* v = argv[i + 1];
    if (k == "--socket") sock = v;
    else if (k == "--device") b.device = std::atoi(v);
    else if (k == "--pci-bus-id") pci = v;  // the GPU by PCI address (HIP and SMI orders differ)
    else if (k == "--gib") gib = std::atof(v);
    else if (k == "--reserve-gib") reserve_gib = std::atof(v);
    else if (k == "--granule-mib") gran_mib = std::strtoull(v, nullptr, 10);
    else if (k == "--wait-s") b.wait_s = std::atof(v);
    else if (k == "--grant-ttl-s") b.grant_ttl_s = std::atof(v);
    else {
      std::fprintf(stderr, "gpushare-hbm-broker: unknown flag %s\n", k.c_str());
      return 2;
    }
  }
  if (sock.empty()) {
    std::fprintf(stderr, "usage: gpushare-hbm-broker --socket PATH [--device N | --pci-bus-id BDF] [--gib N | --reserve-gib N] "
                         "[--granule-mib 1024] [--wait-s 30]\n");
    return 2;
  }
  b.gran = gran_mib << 20;
  if (!pci.empty()) CK(hipDeviceGetByPCIBusId(&b.device, pci.c_str()));
  CK(hipSetDevice(b.device));
  size_t fr = 0, tot = 0;
  CK(hipMemGetInfo(&fr, &tot));
  size_t total = gib > 0 ? size_t(gib * double(1ull << 30))
                         : (fr > size_t(reserve_gib * double(1ull << 30)) ? fr - size_t(reserve_gib * double(1ull << 30)) : 0);
  b.setup(total);
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  signal(SIGPIPE, SIG_IGN);
  int pod_ls = listen_unix(sock, 0666);
  int adm_ls = listen_unix(sock + ".admin", 0600);
  std::printf("{\"ready\": true, \"socket\": \"%s\", \"granules\": %d, \"granule_bytes\": %zu, \"setup_ms\": %.1f}\n",
              sock.c_str(), b.count, b.gran, b.setup_s * 1e3);
  std::fflush(stdout);

  while (!g_stop) {
    std::vector<pollfd> pf{{pod_ls, POLLIN, 0}, {adm_ls, POLLIN, 0}};
    for (auto& kv : b.clients) pf.push_back({kv.first, POLLIN, 0});
    // a retired tenant's references drop when the kernel finishes tearing its process down:
    // look often while granules wait for that, so the next pod's TAKE is not held up
    int r = poll(pf.data(), pf.size(), b.quarantine.empty() ? 100 : 3);
    if (r < 0) continue;
    for (int k = 0; k < 2; ++k)
      if (pf[k].revents & POLLIN) {
        int c = accept4(pf[k].fd, nullptr, nullptr, SOCK_CLOEXEC);
        if (c >= 0) b.clients[c].fd = c, b.clients[c].admin = (k == 1);
      }
    for (size_t k = 2; k < pf.size(); ++k) {
      if (!pf[k].revents) continue;
      int fd = pf[k].fd;
      char buf[512];
      ssize_t n = recv(fd, buf, sizeof buf, 0);
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
    // TAKEs that waited too long are refused (their grant stays for a retry)
    double t = now_s();
    std::vector<int> late;
    for (auto& kv : b.clients)
      if (!kv.second.waiting.empty() && t - kv.second.wait_since > b.wait_s) late.push_back(kv.first);
    for (int fd : late) {
      ++b.timeouts;
      Broker::reply(fd, "ERR timeout\n");
      b.drop(fd);
    }
    if (!b.quarantine.empty() && b.sweep_quarantine()) b.serve_waiting();
    // grants of pods that never started (deleted before admission) do not pile up
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
  unlink(sock.c_str());
  unlink((sock + ".admin").c_str());
  return 0;
}
