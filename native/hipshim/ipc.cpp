// Inter-process sharing of arena memory: hipIpcGetMemHandle / hipIpcOpenMemHandle /
// hipIpcCloseMemHandle, and hipMemGetAddressRange (shim.h lists the units and the lock order).
//
// Arena memory is VMM-mapped granules imported from the broker's dma-bufs, which the runtime's own
// IPC cannot export (hipIpcGetMemHandle fails with hipErrorInvalidValue on MI355X,
// profiles/r6/arena_probe.jsonl): torch.multiprocessing's CUDA tensor sharing, RCCL's P2P buffers
// and serving stacks would break under a grant. So the shim exports them itself (VERDICT r5
// weak 3). The handle names the exporting process, a random secret of it and an export; the
// importer's shim connects to the exporter's abstract unix socket (the pod's network namespace:
// processes of one pod), presents the secret and receives the fds of the granules the allocation
// spans (SCM_RIGHTS), then imports and maps them as the arena does. The secret is the capability,
// as a CUDA IPC handle is one. The fds are not fetched with pidfd_getfd: the pool's kernels run
// Yama ptrace_scope 1, under which a child may not take its parent's fds.
//
// The broker's granules stay referenced while an importer maps them, so the broker's release
// policy ("refs": no dma-buf reference left outside it) keeps them out of the free list until the
// importer closes its mapping or exits, even after the exporter is gone. Imported memory is not
// charged to the importer's quota (it is its exporter's).
#include "shim.h"

#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

namespace gs {
namespace {

constexpr uint32_t kIpcMagic = 0x50495347;  // "GSIP"
struct IpcHandle {
  uint32_t magic;
  uint32_t version;
  int32_t pid;
  uint32_t id;
  uint64_t nonce;
  uint64_t len;    // bytes from the exported pointer to the end of its allocation
  uint64_t delta;  // exported pointer - start of its allocation
  uint8_t pad[24];
};
static_assert(sizeof(IpcHandle) == sizeof(hipIpcMemHandle_t), "IPC handle layout");

struct Export {
  uint32_t id;
  uint64_t off, len;  // the allocation in the arena
};
struct Mapping {
  char* ret;        // what hipIpcOpenMemHandle returned
  char* base;       // the reservation
  uint64_t vsize, len;
  int k, tag;
  bool local;       // this process's own export: nothing mapped
  hipMemGenericAllocationHandle_t* h;
};
constexpr int kMaxExports = 4096, kMaxMappings = 1024;

struct Ipc {
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;  // leaf: exports and mappings
  Export exports[kMaxExports];
  int nexports = 0;
  uint32_t next_id = 1;
  uint64_t nonce = 0;
  int listen_fd = -1;
  bool serving = false;
  Mapping maps[kMaxMappings];
  int nmaps = 0;
  int next_tag = 2;  // 1 is the arena's
  uint64_t served = 0, opened = 0;
};
Ipc g_ipc;

void sock_name(sockaddr_un* sa, socklen_t* len, int pid, uint64_t nonce) {
  memset(sa, 0, sizeof *sa);
  sa->sun_family = AF_UNIX;
  int n = snprintf(sa->sun_path + 1, sizeof sa->sun_path - 1, "gpushare-ipc/%d/%016llx", pid, (unsigned long long)nonce);
  *len = socklen_t(offsetof(sockaddr_un, sun_path) + 1 + size_t(n));
}

uint64_t random64() {
  uint64_t v = 0;
  int fd = open("/dev/urandom", O_RDONLY | O_CLOEXEC);
  if (fd >= 0) {
    if (read(fd, &v, sizeof v) != ssize_t(sizeof v)) v = 0;
    close(fd);
  }
  return v ? v : (mono_ns() ^ (uint64_t(getpid()) << 32)) | 1;
}

bool send_line(int s, const char* line) {
  size_t n = strlen(line);
  return send(s, line, n, MSG_NOSIGNAL) == ssize_t(n);
}

bool read_line(int s, char* buf, size_t cap, int timeout_ms) {
  size_t i = 0;
  while (i + 1 < cap) {
    pollfd p{s, POLLIN, 0};
    if (poll(&p, 1, timeout_ms) <= 0) return false;
    char ch;
    if (recv(s, &ch, 1, 0) != 1) return false;
    if (ch == '\n') break;
    buf[i++] = ch;
  }
  buf[i] = 0;
  return true;
}

bool send_fds(int s, const int* fds, int k) {
  for (int i = 0; i < k; i += 200) {
    int m = k - i < 200 ? k - i : 200;
    char byte = 'f';
    iovec io{&byte, 1};
    alignas(cmsghdr) char ctl[CMSG_SPACE(200 * sizeof(int))];
    msghdr msg;
    memset(&msg, 0, sizeof msg);
    msg.msg_iov = &io;
    msg.msg_iovlen = 1;
    msg.msg_control = ctl;
    msg.msg_controllen = CMSG_SPACE(size_t(m) * sizeof(int));
    cmsghdr* c = CMSG_FIRSTHDR(&msg);
    c->cmsg_level = SOL_SOCKET;
    c->cmsg_type = SCM_RIGHTS;
    c->cmsg_len = CMSG_LEN(size_t(m) * sizeof(int));
    memcpy(CMSG_DATA(c), fds + i, size_t(m) * sizeof(int));
    if (sendmsg(s, &msg, MSG_NOSIGNAL) != 1) return false;
  }
  return true;
}

bool recv_fds(int s, int* fds, int k) {
  int got = 0;
  while (got < k) {
    char byte;
    iovec io{&byte, 1};
    alignas(cmsghdr) char ctl[CMSG_SPACE(200 * sizeof(int))];
    msghdr m;
    memset(&m, 0, sizeof m);
    m.msg_iov = &io;
    m.msg_iovlen = 1;
    m.msg_control = ctl;
    m.msg_controllen = sizeof ctl;
    pollfd p{s, POLLIN, 0};
    if (poll(&p, 1, 5000) <= 0 || recvmsg(s, &m, MSG_CMSG_CLOEXEC) != 1) break;
    cmsghdr* c = CMSG_FIRSTHDR(&m);
    if (!c || c->cmsg_level != SOL_SOCKET || c->cmsg_type != SCM_RIGHTS) break;
    int n = int((c->cmsg_len - CMSG_LEN(0)) / sizeof(int));
    const int* q = reinterpret_cast<const int*>(CMSG_DATA(c));
    for (int i = 0; i < n; ++i) {
      if (got < k) fds[got++] = q[i];
      else close(q[i]);
    }
  }
  if (got == k) return true;
  for (int i = 0; i < got; ++i) close(fds[i]);
  return false;
}

// one request on an accepted connection: "GET <nonce> <id>" -> "OK <gran> <first> <len> <k>" + k fds
void serve_one(int c) {
  char line[128];
  unsigned long long nonce = 0;
  unsigned id = 0;
  if (!read_line(c, line, sizeof line, 2000) || sscanf(line, "GET %llx %u", &nonce, &id) != 2 ||
      nonce != g_ipc.nonce) {
    send_line(c, "ERR handle\n");
    return;
  }
  Arena& a = g_arena;
  int dups[kArenaMaxGranules];
  int k = 0;
  uint64_t gran = 0, first = 0, len = 0;
  pthread_mutex_lock(&a.mu);
  pthread_mutex_lock(&g_ipc.mu);
  const Export* e = nullptr;
  for (int i = 0; i < g_ipc.nexports && !e; ++i)
    if (g_ipc.exports[i].id == id) e = &g_ipc.exports[i];
  if (e && a.state.load() == 1) {
    gran = a.gran;
    int g0 = int(e->off / gran), g1 = int((e->off + e->len - 1) / gran);
    first = e->off - uint64_t(g0) * gran;
    len = e->len;
    for (int gi = g0; gi <= g1 && gi < a.n; ++gi) {
      int d = a.fd[gi] >= 0 ? fcntl(a.fd[gi], F_DUPFD_CLOEXEC, 0) : -1;
      if (d < 0) break;
      dups[k++] = d;
    }
    if (k != g1 - g0 + 1) {
      for (int i = 0; i < k; ++i) close(dups[i]);
      k = -1;
    }
  } else {
    k = -1;
  }
  pthread_mutex_unlock(&g_ipc.mu);
  pthread_mutex_unlock(&a.mu);
  if (k < 0) {
    send_line(c, "ERR gone\n");
    return;
  }
  snprintf(line, sizeof line, "OK %llu %llu %llu %d\n", (unsigned long long)gran, (unsigned long long)first,
           (unsigned long long)len, k);
  if (send_line(c, line)) send_fds(c, dups, k);
  for (int i = 0; i < k; ++i) close(dups[i]);
  pthread_mutex_lock(&g_ipc.mu);
  ++g_ipc.served;
  pthread_mutex_unlock(&g_ipc.mu);
}

void* server(void*) {
  int ls = g_ipc.listen_fd;
  for (;;) {
    int c = accept4(ls, nullptr, nullptr, SOCK_CLOEXEC);
    if (c < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      return nullptr;  // the socket is gone (a forked child's copy, or the process is ending)
    }
    serve_one(c);
    close(c);
  }
}

// the exporter's socket and server thread, at the first export (g_ipc.mu held)
bool ensure_server() {
  if (g_ipc.serving) return true;
  g_ipc.nonce = random64();
  int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_un sa;
  socklen_t len;
  sock_name(&sa, &len, getpid(), g_ipc.nonce);
  if (s < 0 || bind(s, reinterpret_cast<sockaddr*>(&sa), len) != 0 || listen(s, 64) != 0) {
    logf(1, "ipc: cannot listen (%s)", strerror(errno));
    if (s >= 0) close(s);
    return false;
  }
  g_ipc.listen_fd = s;
  pthread_attr_t at;
  pthread_attr_init(&at);
  pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
  pthread_attr_setstacksize(&at, 256 << 10);
  sigset_t all, old;
  sigfillset(&all);
  pthread_sigmask(SIG_BLOCK, &all, &old);
  pthread_t th;
  int rc = pthread_create(&th, &at, server, nullptr);
  pthread_sigmask(SIG_SETMASK, &old, nullptr);
  pthread_attr_destroy(&at);
  if (rc != 0) {
    close(s);
    g_ipc.listen_fd = -1;
    return false;
  }
  g_ipc.serving = true;
  return true;
}

Mapping* mapping_of(const char* p, bool exact) {
  for (int i = 0; i < g_ipc.nmaps; ++i) {
    Mapping& m = g_ipc.maps[i];
    if (exact ? p == m.ret : (p >= m.ret && p < m.ret + m.len)) return &m;
  }
  return nullptr;
}

hipError_t open_remote(void** ptr, const IpcHandle& h) {
  int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_un sa;
  socklen_t len;
  sock_name(&sa, &len, h.pid, h.nonce);
  char line[128];
  unsigned long long gran = 0, first = 0, blen = 0;
  int k = 0;
  if (s < 0 || connect(s, reinterpret_cast<sockaddr*>(&sa), len) != 0) {
    logf(1, "ipc: exporter %d not reachable (%s)", h.pid, strerror(errno));
    if (s >= 0) close(s);
    return hipErrorInvalidValue;
  }
  snprintf(line, sizeof line, "GET %016llx %u\n", (unsigned long long)h.nonce, h.id);
  if (!send_line(s, line) || !read_line(s, line, sizeof line, 5000) ||
      sscanf(line, "OK %llu %llu %llu %d", &gran, &first, &blen, &k) != 4 || k <= 0 || k > kArenaMaxGranules ||
      gran == 0 || first >= gran) {
    logf(1, "ipc: exporter %d refused (%s)", h.pid, line);
    close(s);
    return hipErrorInvalidValue;
  }
  int fds[kArenaMaxGranules];
  bool got = recv_fds(s, fds, k);
  close(s);
  if (!got) return hipErrorInvalidValue;
  auto reserve_f = real_hipMemAddressReserve();
  auto free_f = real_hipMemAddressFree();
  auto un = real_hipMemUnmap();
  auto rel = real_hipMemRelease();
  auto gd = real_hipGetDevice();
  Mapping m;
  memset(&m, 0, sizeof m);
  m.vsize = uint64_t(k) * gran;
  m.k = k;
  m.h = static_cast<hipMemGenericAllocationHandle_t*>(calloc(size_t(k), sizeof(hipMemGenericAllocationHandle_t)));
  int dev = 0;
  hipError_t e = hipErrorInvalidValue;
  {
    Depth d;
    void* base = nullptr;
    if (m.h && reserve_f && gd && gd(&dev) == hipSuccess && reserve_f(&base, m.vsize, 0, nullptr, 0) == hipSuccess) {
      m.base = static_cast<char*>(base);
      pthread_mutex_lock(&g_ipc.mu);
      m.tag = g_ipc.next_tag++;
      pthread_mutex_unlock(&g_ipc.mu);
      int rtv = runtime_version();
      t_import_tag = m.tag;
      int failed = import_and_map(fds, k, m.h, m.base, gran, rtv > 0 && rtv < 70100000);
      t_import_tag = 0;
      if (!failed && set_rw(m.base, m.vsize, dev)) e = hipSuccess;
      if (e != hipSuccess) {
        for (int i = 0; i < k; ++i)
          if (m.h[i]) {
            if (un) (void)un(m.base + uint64_t(i) * gran, gran);
            if (rel) (void)rel(m.h[i]);
          }
        if (rtv > 0 && rtv < 70100000) imports_free(m.tag);
        if (free_f) (void)free_f(m.base, m.vsize);
      }
    }
  }
  for (int i = 0; i < k; ++i) close(fds[i]);
  if (e != hipSuccess) {
    free(m.h);
    logf(1, "ipc: mapping %d granules of exporter %d failed", k, h.pid);
    return e;
  }
  m.ret = m.base + first + h.delta;
  m.len = blen - h.delta;
  pthread_mutex_lock(&g_ipc.mu);
  if (g_ipc.nmaps < kMaxMappings) {
    g_ipc.maps[g_ipc.nmaps++] = m;
    ++g_ipc.opened;
    e = hipSuccess;
  } else {
    e = hipErrorOutOfMemory;
  }
  pthread_mutex_unlock(&g_ipc.mu);
  if (e != hipSuccess) {  // no room to remember it: undo
    Depth d;
    for (int i = 0; i < k; ++i) {
      if (un) (void)un(m.base + uint64_t(i) * gran, gran);
      if (rel) (void)rel(m.h[i]);
    }
    if (free_f) (void)free_f(m.base, m.vsize);
    free(m.h);
    return e;
  }
  *ptr = m.ret;
  logf(2, "ipc: opened %d granules of exporter %d at %p", k, h.pid, m.ret);
  return hipSuccess;
}

void close_mapping(Mapping m) {
  if (m.local) return;
  auto un = real_hipMemUnmap();
  auto rel = real_hipMemRelease();
  auto free_f = real_hipMemAddressFree();
  Depth d;
  if (auto sync = real_hipDeviceSynchronize()) (void)sync();  // nothing may still use it
  uint64_t gran = m.vsize / uint64_t(m.k);
  for (int i = 0; i < m.k; ++i) {
    if (un) (void)un(m.base + uint64_t(i) * gran, gran);
    if (rel && m.h[i]) (void)rel(m.h[i]);
  }
  int rtv = runtime_version();
  if (rtv > 0 && rtv < 70100000) imports_free(m.tag);  // HIP 7.0 keeps them (see kfd.cpp)
  if (free_f) (void)free_f(m.base, m.vsize);
  free(m.h);
}
}  // namespace

void ipc_forget_block(uint64_t off) {
  pthread_mutex_lock(&g_ipc.mu);
  for (int i = 0; i < g_ipc.nexports;)
    if (g_ipc.exports[i].off == off) g_ipc.exports[i] = g_ipc.exports[--g_ipc.nexports];
    else ++i;
  pthread_mutex_unlock(&g_ipc.mu);
}

void ipc_atfork_child() {
  pthread_mutex_init(&g_ipc.mu, nullptr);
  if (g_ipc.listen_fd >= 0) close(g_ipc.listen_fd);
  g_ipc.listen_fd = -1;
  g_ipc.serving = false;
  g_ipc.nexports = 0;
  g_ipc.nmaps = 0;  // the parent's mappings are the parent's
}

}  // namespace gs

using namespace gs;

GS_EXPORT hipError_t hipIpcGetMemHandle(hipIpcMemHandle_t* handle, void* ptr) {
  auto f = real_hipIpcGetMemHandle();
  if (!f) return hipErrorNotInitialized;
  if (!handle || !ptr || t_depth || !arena_configured() || !arena_owns(ptr)) return f(handle, ptr);
  Arena& a = g_arena;
  uint64_t off = uint64_t(static_cast<char*>(ptr) - a.base), start = 0, len = 0;
  hipError_t e = hipErrorInvalidValue;
  pthread_mutex_lock(&a.mu);
  bool live = arena_live_find(off, &start, &len);
  pthread_mutex_lock(&g_ipc.mu);
  if (live && g_ipc.nexports < kMaxExports && ensure_server()) {
    IpcHandle h;
    memset(&h, 0, sizeof h);
    h.magic = kIpcMagic;
    h.version = 1;
    h.pid = getpid();
    h.id = g_ipc.next_id++;
    h.nonce = g_ipc.nonce;
    h.len = start + len - off;
    h.delta = off - start;
    g_ipc.exports[g_ipc.nexports++] = {h.id, start, len};
    memcpy(handle, &h, sizeof h);
    e = hipSuccess;
  }
  pthread_mutex_unlock(&g_ipc.mu);
  pthread_mutex_unlock(&a.mu);
  if (e != hipSuccess) logf(1, "ipc: no handle for %p (%s)", ptr, live ? "no room" : "not a live allocation");
  return e;
}

GS_EXPORT hipError_t hipIpcOpenMemHandle(void** ptr, hipIpcMemHandle_t handle, unsigned int flags) {
  auto f = real_hipIpcOpenMemHandle();
  IpcHandle h;
  memcpy(&h, &handle, sizeof h);
  if (h.magic != kIpcMagic || h.version != 1) return f ? f(ptr, handle, flags) : hipErrorNotInitialized;
  if (!ptr) return hipErrorInvalidValue;
  if (h.pid == getpid()) {  // this process's own export: the memory is mapped here already
    Arena& a = g_arena;
    hipError_t e = hipErrorInvalidValue;
    pthread_mutex_lock(&a.mu);
    pthread_mutex_lock(&g_ipc.mu);
    for (int i = 0; i < g_ipc.nexports; ++i)
      if (g_ipc.exports[i].id == h.id && h.nonce == g_ipc.nonce && g_ipc.nmaps < kMaxMappings) {
        Mapping m;
        memset(&m, 0, sizeof m);
        m.ret = a.base + g_ipc.exports[i].off + h.delta;
        m.len = h.len;
        m.local = true;
        g_ipc.maps[g_ipc.nmaps++] = m;
        *ptr = m.ret;
        e = hipSuccess;
        break;
      }
    pthread_mutex_unlock(&g_ipc.mu);
    pthread_mutex_unlock(&a.mu);
    return e;
  }
  return open_remote(ptr, h);
}

GS_EXPORT hipError_t hipIpcCloseMemHandle(void* ptr) {
  auto f = real_hipIpcCloseMemHandle();
  pthread_mutex_lock(&g_ipc.mu);
  Mapping* m = mapping_of(static_cast<char*>(ptr), true);
  Mapping copy;
  if (m) {
    copy = *m;
    *m = g_ipc.maps[--g_ipc.nmaps];
  }
  pthread_mutex_unlock(&g_ipc.mu);
  if (!m) return f ? f(ptr) : hipErrorNotInitialized;
  close_mapping(copy);
  return hipSuccess;
}

// The allocation a pointer lies in. For arena memory the runtime would answer with the granule's
// mapping (1 GiB), not the program's allocation; the shim answers with the allocation, as for
// any hipMalloc pointer. IPC mappings answer with what was opened.
GS_EXPORT hipError_t hipMemGetAddressRange(hipDeviceptr_t* base, size_t* size, hipDeviceptr_t ptr) {
  auto f = real_hipMemGetAddressRange();
  if (!f) return hipErrorNotInitialized;
  if (ptr && !t_depth) {
    if (arena_configured() && arena_owns(ptr)) {
      Arena& a = g_arena;
      uint64_t start = 0, len = 0;
      pthread_mutex_lock(&a.mu);
      bool live = arena_live_find(uint64_t(static_cast<char*>(ptr) - a.base), &start, &len);
      pthread_mutex_unlock(&a.mu);
      if (!live) return hipErrorNotFound;
      if (base) *base = a.base + start;
      if (size) *size = size_t(len);
      return hipSuccess;
    }
    pthread_mutex_lock(&g_ipc.mu);
    Mapping* m = mapping_of(static_cast<char*>(ptr), false);
    char* r = m ? m->ret : nullptr;
    uint64_t len = m ? m->len : 0;
    pthread_mutex_unlock(&g_ipc.mu);
    if (m) {
      if (base) *base = r;
      if (size) *size = size_t(len);
      return hipSuccess;
    }
  }
  return f(base, size, ptr);
}

// exports made, requests served, mappings opened (ever) and open now
GS_EXPORT int gpushare_shim_ipc_stats(uint64_t* exports, uint64_t* served, uint64_t* opened, uint64_t* open_now) {
  pthread_mutex_lock(&g_ipc.mu);
  if (exports) *exports = g_ipc.next_id - 1;
  if (served) *served = g_ipc.served;
  if (opened) *opened = g_ipc.opened;
  if (open_now) *open_now = uint64_t(g_ipc.nmaps);
  pthread_mutex_unlock(&g_ipc.mu);
  return 1;
}
