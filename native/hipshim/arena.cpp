// The HBM-broker arena of the quota shim (shim.h lists the units and the lock order).
//
// GPUSHARE_HBM_BROKER=<socket> + GPUSHARE_HBM_TOKEN=<token>: the pod's HBM comes from the node's
// HBM broker (native/hbmbroker) instead of fresh driver allocations, so it never waits for
// amdgpu's wipe of a retired pod's memory. At the first allocation the shim takes its grant (the
// fds of its granules, and only those), imports and maps them contiguously, and serves
// allocations from that range. The broker connection stays open for the process lifetime: its
// end returns the granules (scrubbed) to the broker. gpushare_shim_arena_release() hands them
// back early, once nothing in the arena is live.
//
// The whole quota is usable. The grant is a share of the quota; the address
// range is reserved for the whole quota (the broker's "limit"). An allocation the arena cannot
// serve waits for granules the broker still owes (a streaming TAKE), then asks for granules
// beyond the grant (EXTEND: the broker lends granules no grant claims, up to the limit), and
// otherwise goes to the driver, charged to the same ledger. hipMemGetInfo (api.cpp) reports the
// arena's rest plus what the pod can still obtain: the quota's rest, bounded by what the driver
// has free plus what the broker could lend it (AVAIL).
//
// Fast exit: a pod stopped the way the kubelet stops it (SIGTERM, default handler) or that just
// exits never calls gpushare_shim_arena_release(). The kernel then releases the process's KFD
// imports of its granules only when it has torn the process down, 300-380 ms after the signal on
// MI355X (profiles/r6/arena_probe.jsonl), and the broker cannot lend them before. So at SIGTERM
// (when the program has no handler of its own) and at the end of a normal exit, the shim destroys
// the process's queues the way the kernel does at exit — nothing on the GPU can touch the
// process's memory after that — and frees the imports itself. GPUSHARE_SHIM_FAST_EXIT=0 leaves it
// to the kernel.
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
#include <time.h>
#include <unistd.h>

namespace gs {

Arena g_arena;
int g_dev = 0;

namespace {
// where a TAKE's time went (ns): connecting to the broker, waiting for its answer, importing and
// mapping the granules (gpushare_shim_arena_timing); then, for a streaming TAKE, allocations that
// waited for owed granules, importing and mapping those, and MORE messages received
uint64_t g_take_connect_ns = 0, g_take_wait_ns = 0, g_take_map_ns = 0;
uint64_t g_more_wait_ns = 0, g_more_map_ns = 0, g_more_msgs = 0, g_more_waits = 0;
uint64_t g_take_first = 0, g_take_reserve_ns = 0, g_take_access_ns = 0;  // the TAKE's first batch
uint64_t g_first_import_ns = 0, g_first_map_ns = 0;  // the process's first granule
uint64_t g_take_header_ns = 0;                       // TAKE sent -> the broker's answer line
uint64_t g_extends = 0, g_extended = 0, g_driver_allocs = 0, g_driver_bytes = 0;
// where the last arena release spent its time (ns): device sync, unmaps, address free, handle
// releases, the KFD frees of kept imports (gpushare_shim_arena_release_timing)
uint64_t g_rel_ns[5];

bool recv_line_ms(int s, char* buf, size_t cap, int timeout_ms) {
  size_t i = 0;
  while (i + 1 < cap) {
    if (timeout_ms >= 0) {
      pollfd p{s, POLLIN, 0};
      if (poll(&p, 1, timeout_ms) <= 0) return false;
    }
    char ch;
    ssize_t r = recv(s, &ch, 1, 0);
    if (r <= 0) return false;
    if (ch == '\n') break;
    buf[i++] = ch;
  }
  buf[i] = 0;
  return true;
}

bool recv_line(int s, char* buf, size_t cap) { return recv_line_ms(s, buf, cap, -1); }

// fds of one SCM_RIGHTS message into out[*got...]
bool recv_fd_batch(int s, int* out, int* got, int want) {
  char byte;
  iovec io{&byte, 1};
  alignas(cmsghdr) char ctl[CMSG_SPACE(200 * sizeof(int))];
  msghdr m;
  memset(&m, 0, sizeof m);
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  if (recvmsg(s, &m, MSG_CMSG_CLOEXEC) != 1) return false;
  cmsghdr* c = CMSG_FIRSTHDR(&m);
  if (!c || c->cmsg_level != SOL_SOCKET || c->cmsg_type != SCM_RIGHTS) return false;
  int k = int((c->cmsg_len - CMSG_LEN(0)) / sizeof(int));
  const int* p = reinterpret_cast<const int*>(CMSG_DATA(c));
  for (int i = 0; i < k; ++i) {
    if (*got < want) out[(*got)++] = p[i];
    else close(p[i]);
  }
  return true;
}

bool recv_fds(int s, int* fds, int k) {
  int got = 0;
  while (got < k)
    if (!recv_fd_batch(s, fds, &got, k)) {
      for (int i = 0; i < got; ++i) close(fds[i]);
      return false;
    }
  return true;
}

// ---- the allocator: free extents and live blocks, both sorted by offset (g_arena.mu held) ----
int ext_lower(uint64_t off) {  // first extent at or after off
  Arena& a = g_arena;
  int lo = 0, hi = a.next;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (a.ext[mid].off < off) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

int live_lower(uint64_t off) {  // first live block at or after off
  Arena& a = g_arena;
  int lo = 0, hi = a.nlive;
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (a.live[mid].off < off) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

bool live_put(uint64_t off, uint64_t len) {
  Arena& a = g_arena;
  if (a.nlive >= kArenaMaxLive) return false;
  int i = live_lower(off);
  memmove(&a.live[i + 1], &a.live[i], sizeof(Ext) * size_t(a.nlive - i));
  a.live[i] = {off, len};
  ++a.nlive;
  return true;
}

bool live_take(uint64_t off, uint64_t* len) {
  Arena& a = g_arena;
  int i = live_lower(off);
  if (i >= a.nlive || a.live[i].off != off) return false;
  *len = a.live[i].len;
  memmove(&a.live[i], &a.live[i + 1], sizeof(Ext) * size_t(a.nlive - i - 1));
  --a.nlive;
  return true;
}

// take [start, start + len) out of free extent i (it lies inside it)
bool arena_carve(int i, uint64_t start, uint64_t len) {
  Arena& a = g_arena;
  Ext e = a.ext[i];
  uint64_t head = start - e.off, tail = e.off + e.len - (start + len);
  if (head && tail && a.next >= kArenaMaxExt) return false;
  if (!live_put(start, len)) return false;
  if (head && tail) {  // split in two: shift the rest up by one
    memmove(&a.ext[i + 2], &a.ext[i + 1], sizeof(Ext) * (a.next - i - 1));
    a.ext[i] = {e.off, head};
    a.ext[i + 1] = {start + len, tail};
    ++a.next;
  } else if (head) {
    a.ext[i] = {e.off, head};
  } else if (tail) {
    a.ext[i] = {start + len, tail};
  } else {
    memmove(&a.ext[i], &a.ext[i + 1], sizeof(Ext) * (a.next - i - 1));
    --a.next;
  }
  a.used += len;
  return true;
}

// [off, off + len) is free again: into the sorted extent list, joined with its neighbours
void ext_insert(uint64_t off, uint64_t len) {
  Arena& a = g_arena;
  int lo = ext_lower(off);
  bool join_prev = lo > 0 && a.ext[lo - 1].off + a.ext[lo - 1].len == off;
  bool join_next = lo < a.next && off + len == a.ext[lo].off;
  if (join_prev && join_next) {
    a.ext[lo - 1].len += len + a.ext[lo].len;
    memmove(&a.ext[lo], &a.ext[lo + 1], sizeof(Ext) * (a.next - lo - 1));
    --a.next;
  } else if (join_prev) {
    a.ext[lo - 1].len += len;
  } else if (join_next) {
    a.ext[lo].off = off;
    a.ext[lo].len += len;
  } else if (a.next < kArenaMaxExt) {
    memmove(&a.ext[lo + 1], &a.ext[lo], sizeof(Ext) * (a.next - lo));
    a.ext[lo] = {off, len};
    ++a.next;
  }  // else: the extent list is full and these bytes stay unusable until release (never seen)
}

uint64_t align_of(uint64_t size) { return size >= (2ull << 20) ? (2ull << 20) : 4096; }

// ---- the broker connection ----------------------------------------------------------------
// the broker will send no more (it went away, ended the stream, or sent something else): the
// grant shrinks to what was delivered, and the ledger with it (g_arena.mu held)
void arena_stream_end(const char* why) {
  Arena& a = g_arena;
  logf(1, "hbm broker: stream ended (%s) at %d of %d granules", why, a.n, a.total);
  uint64_t owed = uint64_t(a.total - a.n) * a.gran;
  a.total = a.n;
  a.size -= owed;
  if (a.charged) uncharge(owed);
}

// a line from the broker outside a reply: END (revoked, or owed granules cancelled) — no more
// granules of any kind. true if it was one (the caller reads on)
bool broker_notice(const char* line) {
  Arena& a = g_arena;
  if (strcmp(line, "END") != 0) return false;
  if (a.n < a.total) arena_stream_end("END");
  a.ended = true;
  return true;
}

// unmap and release whatever of the arena is mapped (g_arena.mu held)
void arena_unmap_locked() {
  Arena& a = g_arena;
  Depth d;
  uint64_t t0 = mono_ns();
  if (auto dev_sync = real_hipDeviceSynchronize()) (void)dev_sync();
  uint64_t t1 = mono_ns(), t2 = t1, t3 = t1;
  if (a.base) {
    // one unmap per mapping: HIP unmaps one handle's mapping per call. Unmapping the whole range
    // at once failed, and the imported handles then stayed mapped, keeping the broker's granules
    // referenced until this process was torn down (tools/diag/dmabuf_ref_probe.cpp: with a
    // per-mapping unmap and the release the references go at once)
    if (auto un = real_hipMemUnmap()) {
      int bad = 0;
      for (int i = 0; i < a.n; ++i)
        bad += un(a.base + uint64_t(i) * a.gran, a.gran) != hipSuccess;
      if (bad) logf(1, "hbm broker: %d of %d granule unmaps failed", bad, a.n);
    }
    t2 = mono_ns();
    if (auto fr = real_hipMemAddressFree()) (void)fr(a.base, a.vsize);
    t3 = mono_ns();
  }
  if (auto rel = real_hipMemRelease())
    for (int i = 0; i < a.n; ++i)
      if (a.h[i]) (void)rel(a.h[i]);
  for (int i = 0; i < a.n; ++i)
    if (a.fd[i] >= 0) {
      close(a.fd[i]);
      a.fd[i] = -1;
    }
  uint64_t t4 = mono_ns();
  g_rel_ns[0] = t1 - t0;
  g_rel_ns[1] = t2 - t1;
  g_rel_ns[2] = t3 - t2;
  g_rel_ns[3] = t4 - t3;
  g_rel_ns[4] = 0;
  a.n = a.total = 0;
  a.base = nullptr;
}

// ---- fast exit ----------------------------------------------------------------------------------
int g_exit_pipe[2] = {-1, -1};
struct sigaction g_prev_term;
std::atomic<bool> g_fast_exit_armed{false}, g_fast_exit_done{false};

void fast_release(const char* why) {
  if (g_fast_exit_done.exchange(true)) return;
  uint64_t t0 = mono_ns();
  int q = queues_destroy_all();
  int m = imports_free_all_unlocked();
  // the granule fds this process keeps for IPC exports are references of their own: without
  // closing them the broker sees the granules held until the kernel closes the fd table, at the
  // very end of the teardown (measured: 164 ms after SIGTERM, the imports long freed)
  int c = 0;
  for (int i = 0; i < kArenaMaxGranules; ++i) {
    int fd = g_arena.fd[i];
    if (fd >= 0) {
      g_arena.fd[i] = -1;
      close(fd);
      ++c;
    }
  }
  int s = g_arena.sock;
  if (s >= 0) shutdown(s, SHUT_RDWR);  // the broker sees the connection end: the granules are back
  logf(1, "fast exit (%s): %d queues destroyed, %d imports freed, %d granule fds closed in %.3f ms", why, q, m, c,
       (mono_ns() - t0) / 1e6);
}

void on_sigterm(int) {
  char b = 'T';
  ssize_t r = write(g_exit_pipe[1], &b, 1);
  (void)r;
}

void* fast_exit_thread(void*) {
  char b;
  for (;;) {
    ssize_t r = read(g_exit_pipe[0], &b, 1);
    if (r == 1) break;
    if (r < 0 && errno == EINTR) continue;
    return nullptr;  // the pipe is gone (a forked child's copy): nothing to do
  }
  fast_release("SIGTERM");
  // then the signal's default action, as if the shim had never been there
  signal(SIGTERM, SIG_DFL);
  kill(getpid(), SIGTERM);
  usleep(200 * 1000);
  _exit(128 + SIGTERM);  // SIGTERM blocked in every thread: end the same way
  return nullptr;
}

// armed at the arena's TAKE, when the program has left SIGTERM to its default action
void fast_exit_arm() {
  if (!env_u64("GPUSHARE_SHIM_FAST_EXIT", 1) || g_fast_exit_armed.exchange(true)) return;
  struct sigaction cur;
  if (sigaction(SIGTERM, nullptr, &cur) != 0 || (cur.sa_flags & SA_SIGINFO) || cur.sa_handler != SIG_DFL) return;
  if (pipe2(g_exit_pipe, O_CLOEXEC) != 0) return;
  pthread_attr_t at;
  pthread_attr_init(&at);
  pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
  pthread_attr_setstacksize(&at, 64 << 10);
  pthread_t th;
  sigset_t all, old;
  sigfillset(&all);
  pthread_sigmask(SIG_BLOCK, &all, &old);  // the thread takes no signals: the handler may run anywhere else
  int rc = pthread_create(&th, &at, fast_exit_thread, nullptr);
  pthread_sigmask(SIG_SETMASK, &old, nullptr);
  pthread_attr_destroy(&at);
  if (rc != 0) {
    close(g_exit_pipe[0]);
    close(g_exit_pipe[1]);
    g_exit_pipe[0] = g_exit_pipe[1] = -1;
    return;
  }
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_sigterm;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESTART;
  sigaction(SIGTERM, &sa, &g_prev_term);
  logf(2, "fast exit armed");
}

// the end of a normal exit: after the runtime's own teardown (this library was loaded first, so
// its destructor runs last)
__attribute__((destructor)) void fast_exit_at_fini() {
  if (g_arena.state.load() != 1 || !env_u64("GPUSHARE_SHIM_FAST_EXIT", 1)) return;
  fast_release("exit");
}

// A forked child shares none of this: its copy of the broker connection, the granule fds and the
// fast-exit pipe would keep the parent's granules referenced (or end the parent at the child's
// SIGTERM). The child allocates from the driver.
void arena_atfork_child() {
  Arena& a = g_arena;
  pthread_mutex_init(&a.mu, nullptr);
  pthread_cond_init(&a.cv, nullptr);
  if (a.state.load() == 1 || a.sock >= 0) {
    for (int i = 0; i < kArenaMaxGranules; ++i)
      if (a.fd[i] >= 0) {
        close(a.fd[i]);
        a.fd[i] = -1;
      }
    if (a.sock >= 0) close(a.sock);
    a.sock = -1;
    a.state.store(-1);
  }
  a.reading = false;
  if (g_exit_pipe[0] >= 0) {
    struct sigaction cur;
    if (sigaction(SIGTERM, nullptr, &cur) == 0 && cur.sa_handler == on_sigterm) sigaction(SIGTERM, &g_prev_term, nullptr);
    close(g_exit_pipe[0]);
    close(g_exit_pipe[1]);
    g_exit_pipe[0] = g_exit_pipe[1] = -1;
  }
  g_fast_exit_armed.store(false);
  g_fast_exit_done.store(true);  // nothing of the parent's to release here
  ipc_atfork_child();
}

__attribute__((constructor)) void arena_register_atfork() {
  for (auto& f : g_arena.fd) f = -1;
  pthread_atfork(nullptr, nullptr, arena_atfork_child);
}

// called with g_arena.mu held, at the first allocation
void arena_take() {
  Arena& a = g_arena;
  (void)enabled();  // the shim's own init first (log level, quota): the arena is charged below
  a.state.store(-1, std::memory_order_relaxed);
  const char* path = getenv("GPUSHARE_HBM_BROKER");
  const char* tok = getenv("GPUSHARE_HBM_TOKEN");
  int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_un sa;
  memset(&sa, 0, sizeof sa);
  sa.sun_family = AF_UNIX;
  snprintf(sa.sun_path, sizeof sa.sun_path, "%s", path);
  char line[256];
  int fds[kArenaMaxGranules];
  int got = 0;
  unsigned long long want = 0, gran = 0, total = 0, limit = 0;
  int dev = 0;
  // streaming (the default): the broker answers at once with what is free and sends the rest as
  // it comes back; GPUSHARE_HBM_STREAM=0 waits for the whole grant in one answer
  bool stream = env_u64("GPUSHARE_HBM_STREAM", 1) != 0;
  auto import_f = real_hipMemImportFromShareableHandle();
  auto reserve_f = real_hipMemAddressReserve();
  auto map_f = real_hipMemMap();
  auto access_f = real_hipMemSetAccess();
  auto getdev_f = real_hipGetDevice();
  uint64_t t_start = mono_ns(), t_conn = 0, t_fds = 0;
  if (s < 0 || !import_f || !reserve_f || !map_f || !access_f || !getdev_f) goto fail;
  {
    // the broker may not be listening yet (a node booting, a broker restarting): its socket is
    // missing or refuses; retry for GPUSHARE_HBM_WAIT_S (default 15 s), then use the driver
    double wait_s = 15.0;
    if (const char* w = getenv("GPUSHARE_HBM_WAIT_S")) wait_s = atof(w);
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    bool logged = false;
    while (connect(s, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
      int err = errno;
      clock_gettime(CLOCK_MONOTONIC, &t1);
      double el = double(t1.tv_sec - t0.tv_sec) + double(t1.tv_nsec - t0.tv_nsec) * 1e-9;
      if ((err != ENOENT && err != ECONNREFUSED && err != EAGAIN) || el >= wait_s) {
        logf(1, "hbm broker %s: cannot connect (%s) after %.1f s: allocating from the driver", path, strerror(err), el);
        goto fail;
      }
      if (!logged) logf(1, "hbm broker %s: not there yet (%s); waiting up to %.0f s", path, strerror(err), wait_s);
      logged = true;
      timespec nap{0, 50 * 1000 * 1000};
      nanosleep(&nap, nullptr);
      close(s);  // a fresh socket per attempt
      s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
      if (s < 0) goto fail;
    }
  }
  t_conn = mono_ns();
  {
    int n = snprintf(line, sizeof line, stream ? "TAKE %s STREAM\n" : "TAKE %s\n", tok);
    if (send(s, line, n, MSG_NOSIGNAL) != n) goto fail;
  }
  {
    line[0] = 0;
    bool got_line = recv_line(s, line, sizeof line);
    g_take_header_ns = mono_ns() - t_conn;
    int k = got_line ? sscanf(line, "FDS %llu %llu %llu %llu", &want, &gran, &total, &limit) : 0;
    if (k == 2) total = want;
    if (k < 4) limit = total;
    if (k < 2 || total == 0 || want > total || total > (unsigned long long)kArenaMaxGranules || gran == 0) {
      logf(1, "hbm broker %s refused the grant: %s", path, line);
      goto fail;
    }
    if (limit < total) limit = total;
    if (limit > (unsigned long long)kArenaMaxGranules) limit = kArenaMaxGranules;
  }
  {
    uint64_t t_h = mono_ns();
    int batches = 0;
    while (got < (int)want) {
      if (!recv_fd_batch(s, fds, &got, (int)want)) goto fail;
      ++batches;
    }
    t_fds = mono_ns();
    timespec w;
    clock_gettime(CLOCK_REALTIME, &w);
    logf(1, "hbm broker: answer after %.3f ms; %d of %llu granules' fds in %d message(s), %.3f ms; at %.6f",
         g_take_header_ns / 1e6, got, total, batches, (t_fds - t_h) / 1e6, double(w.tv_sec) + w.tv_nsec * 1e-9);
  }
  {
    Depth d;
    if (getdev_f(&dev) != hipSuccess) goto fail;
    // How hipMemImportFromShareableHandle reads a POSIX fd differs by runtime: HIP 7.0 (the one
    // PyTorch bundles, 7.0.51831) reads it through the osHandle pointer and crashes on a bare
    // value; 7.1 and later take the fd as the pointer's value and refuse an address
    // (profiles/r4/vmm_import_semantics.json). Keyed on the runtime's version, not on errors.
    int rtv = runtime_version();
    bool by_address = rtv > 0 && rtv < 70100000;
    logf(1, "hbm broker: runtime %d: fds imported by %s", rtv, by_address ? "address" : "value");
    void* base = nullptr;
    uint64_t vsize = limit * gran;  // the whole quota: granules beyond the grant map after it
    uint64_t t_r = mono_ns();
    // aligned to the granule (GPUSHARE_ARENA_ALIGN_MIB overrides; 0 = the runtime's default), so
    // the GPU's page tables can map each granule with the largest fragments its pages allow
    uint64_t align = env_u64("GPUSHARE_ARENA_ALIGN_MIB", gran >> 20) << 20;
    if (reserve_f(&base, vsize, align, nullptr, 0) != hipSuccess &&
        (align == 0 || reserve_f(&base, vsize, 0, nullptr, 0) != hipSuccess))
      goto fail;
    g_take_reserve_ns = mono_ns() - t_r;
    g_take_first = uint64_t(got);
    logf(2, "hbm broker: reserved %p + %llu", base, (unsigned long long)vsize);
    int failed = import_and_map(fds, got, a.h, static_cast<char*>(base), gran, by_address);
    a.n = got;  // (released at a failure: the ones imported)
    for (int i = 0; i < got; ++i) {
      a.fd[i] = fds[i];  // kept: IPC exports send them (ipc.cpp)
      fds[i] = -1;
    }
    a.base = static_cast<char*>(base);
    a.vsize = vsize;
    a.gran = gran;
    if (failed) {
      logf(1, "hbm broker: import/map of granule %d failed", failed - 1);
      arena_unmap_locked();
      goto fail;  // the broker reclaims at close
    }
    logf(2, "hbm broker: %d granules imported and mapped", got);
    uint64_t t_a = mono_ns();
    if (got && !set_rw(static_cast<char*>(base), uint64_t(got) * gran, dev)) {
      arena_unmap_locked();
      goto fail;
    }
    g_take_access_ns = mono_ns() - t_a;
    a.size = total * gran;
    a.total = int(total);
    a.limit = int(limit);
    a.by_address = by_address;
    a.rt_version = rtv;
    g_dev = dev;
  }
  // the arena counts against the pod's quota like any other HBM it holds: what the runtime
  // still takes from the driver (code objects, scratch) is charged on top of it
  if (enabled() && !charge(a.size)) {
    logf(1, "hbm broker: arena of %llu bytes exceeds the quota (%llu): not used",
         (unsigned long long)a.size, (unsigned long long)g.quota.load());
    arena_unmap_locked();
    goto fail;
  }
  a.charged = enabled();
  a.ext = static_cast<Ext*>(calloc(kArenaMaxExt, sizeof(Ext)));
  a.live = static_cast<Ext*>(calloc(kArenaMaxLive, sizeof(Ext)));
  if (!a.ext || !a.live) goto fail;
  a.ext[0] = {0, uint64_t(a.n) * a.gran};
  a.next = a.n ? 1 : 0;
  a.nlive = 0;
  a.sock = s;
  a.ended = false;
  g_take_connect_ns = t_conn - t_start;
  g_take_wait_ns = t_fds - t_conn;
  g_take_map_ns = mono_ns() - t_fds;
  a.state.store(1, std::memory_order_release);  // base/size published before the state
  logf(1, "hbm broker: %d of %d granules of %llu bytes mapped at %p (limit %d)", a.n, a.total, gran, a.base, a.limit);
  fast_exit_arm();
  return;
fail:
  for (int i = 0; i < got; ++i)
    if (fds[i] >= 0) close(fds[i]);
  if (a.base || a.n) arena_unmap_locked();
  if (a.charged) uncharge(a.size);
  a.charged = false;
  if (s >= 0) close(s);
}

// receive one batch of owed granules (MORE) if it arrives within `wait_ms` (0: only one already
// there); true if the arena grew (g_arena.mu held; the caller owns the socket)
bool more_locked_inner(int wait_ms) {
  Arena& a = g_arena;
  if (a.n >= a.total || a.sock < 0) return false;
  pollfd p{a.sock, POLLIN, 0};
  uint64_t t0 = mono_ns();
  int r = poll(&p, 1, wait_ms);
  if (wait_ms > 0) g_more_wait_ns += mono_ns() - t0;
  if (r <= 0) return false;
  char line[128];
  line[0] = 0;
  unsigned long long k = 0, gran = 0;
  if (!recv_line(a.sock, line, sizeof line)) {
    arena_stream_end("connection closed");
    a.ended = true;
    return false;
  }
  if (broker_notice(line)) return false;
  if (sscanf(line, "MORE %llu %llu", &k, &gran) != 2 || gran != a.gran || k == 0 ||
      k > (unsigned long long)(a.total - a.n)) {
    arena_stream_end(line);
    a.ended = true;
    return false;
  }
  uint64_t t1 = mono_ns();
  int fds[kArenaMaxGranules];
  if (!recv_fds(a.sock, fds, int(k))) {
    arena_stream_end("fds lost");
    a.ended = true;
    return false;
  }
  Depth d;
  char* at = a.base + uint64_t(a.n) * a.gran;
  int failed = import_and_map(fds, int(k), a.h + a.n, at, a.gran, a.by_address);
  if (failed || !set_rw(at, k * a.gran, g_dev)) {
    // keep none of this batch: what was mapped goes, the handles are released
    auto un = real_hipMemUnmap();
    auto rel = real_hipMemRelease();
    for (int i = 0; i < int(k); ++i) {
      if (a.h[a.n + i]) {
        if (un) (void)un(at + uint64_t(i) * a.gran, a.gran);
        if (rel) (void)rel(a.h[a.n + i]);
        a.h[a.n + i] = nullptr;
      }
      close(fds[i]);
    }
    arena_stream_end("import/map failed");
    a.ended = true;
    return false;
  }
  for (int i = 0; i < int(k); ++i) a.fd[a.n + i] = fds[i];
  ext_insert(uint64_t(a.n) * a.gran, k * a.gran);
  a.n += int(k);
  ++g_more_msgs;
  g_more_map_ns += mono_ns() - t1;
  logf(2, "hbm broker: %d more granules, %d of %d mapped", int(k), a.n, a.total);
  return true;
}

// How much room the arena's free tail lacks for an allocation of `size` (0: it fits there).
uint64_t tail_shortfall(uint64_t size) {
  Arena& a = g_arena;
  uint64_t end = uint64_t(a.n) * a.gran, align = align_of(size), len = (size + 4095) & ~uint64_t(4095);
  if (a.next > 0) {
    Ext e = a.ext[a.next - 1];
    if (e.off + e.len == end) {
      uint64_t start = (e.off + align - 1) & ~(align - 1);
      return start + len > end ? start + len - end : 0;
    }
  }
  return len;
}
}  // namespace

bool arena_configured() {
  static std::atomic<int> c{-1};
  int v = c.load(std::memory_order_relaxed);
  if (v < 0) {
    v = getenv("GPUSHARE_HBM_BROKER") && getenv("GPUSHARE_HBM_TOKEN") ? 1 : 0;
    c.store(v, std::memory_order_relaxed);
  }
  return v == 1;
}

int runtime_version() {
  static std::atomic<int> v{-1};
  int r = v.load(std::memory_order_relaxed);
  if (r < 0) {
    auto f = real_hipRuntimeGetVersion();
    Depth d;
    if (!f || f(&r) != hipSuccess) r = 0;
    v.store(r, std::memory_order_relaxed);
  }
  return r;
}

// import fds[0..k) and map granule i at base + i * gran; h[i] set for each one imported (nullptr
// otherwise). Returns 0, or the failed granule + 1. One thread: HIP 7.x's hipMemMap into one
// reservation from several threads at once failed (round 5, bench with 4 mapping threads: an
// allocation in the pod then saw hipErrorInvalidValue)
int import_and_map(int* fds, int k, hipMemGenericAllocationHandle_t* h, char* base, uint64_t gran, bool by_address) {
  auto import_f = real_hipMemImportFromShareableHandle();
  auto map_f = real_hipMemMap();
  for (int i = 0; i < k; ++i) h[i] = nullptr;
  if (!import_f || !map_f) return k > 0 ? 1 : 0;
  Depth d;
  int tag = t_import_tag;
  for (int i = 0; i < k; ++i) {
    uint64_t t0 = mono_ns();
    t_import_tag = tag ? tag : kArenaImportTag;
    hipError_t e = by_address ? import_f(&h[i], &fds[i], hipMemHandleTypePosixFileDescriptor)
                              : import_f(&h[i], reinterpret_cast<void*>(static_cast<intptr_t>(fds[i])),
                                         hipMemHandleTypePosixFileDescriptor);
    t_import_tag = tag;
    uint64_t t1 = mono_ns();
    if (e != hipSuccess) {
      h[i] = nullptr;
      return i + 1;
    }
    e = map_f(base + uint64_t(i) * gran, gran, 0, h[i], 0);
    if (!g_first_import_ns) {  // the process's first import and map (the runtime's one-time work)
      g_first_import_ns = t1 - t0;
      g_first_map_ns = mono_ns() - t1;
    }
    if (e != hipSuccess) return i + 1;
  }
  return 0;
}

// read-write for device `dev`
bool set_rw(char* va, uint64_t len, int dev) {
  hipMemAccessDesc acc;
  memset(&acc, 0, sizeof acc);
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = dev;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  auto f = real_hipMemSetAccess();
  Depth d;
  return f && f(va, len, &acc, 1) == hipSuccess;
}

void arena_ensure() {
  Arena& a = g_arena;
  if (a.state.load(std::memory_order_acquire) != 0) return;
  pthread_mutex_lock(&a.mu);
  if (a.state == 0) arena_take();
  pthread_mutex_unlock(&a.mu);
}

bool arena_owns(const void* p) {
  Arena& a = g_arena;
  const char* c = static_cast<const char*>(p);
  return a.state.load(std::memory_order_acquire) == 1 && c >= a.base && c < a.base + a.vsize;
}

// first fit; large blocks on 2 MiB boundaries (the CDNA4 TLB fragment), small ones on 4 KiB
bool arena_alloc(uint64_t size, void** ptr) {
  Arena& a = g_arena;
  uint64_t align = align_of(size);
  uint64_t len = (size + 4095) & ~uint64_t(4095);
  for (int i = 0; i < a.next; ++i) {
    Ext e = a.ext[i];
    uint64_t start = (e.off + align - 1) & ~(align - 1);
    if (start + len > e.off + e.len) continue;
    if (!arena_carve(i, start, len)) return false;
    *ptr = a.base + start;
    return true;
  }
  return false;
}

// whether an allocation of `size` bytes would find room now (first fit, as arena_alloc)
bool arena_fits(uint64_t size) {
  Arena& a = g_arena;
  uint64_t align = align_of(size);
  uint64_t len = (size + 4095) & ~uint64_t(4095);
  for (int i = 0; i < a.next; ++i) {
    Ext e = a.ext[i];
    uint64_t start = (e.off + align - 1) & ~(align - 1);
    if (start + len <= e.off + e.len) return true;
  }
  return false;
}

// one whole granule (granule-aligned in the arena), last fit: the VMM windows' slots take
// granules from the top while hipMalloc blocks fill from the bottom
bool arena_take_granule(uint64_t* off) {
  Arena& a = g_arena;
  for (int i = a.next - 1; i >= 0; --i) {
    Ext e = a.ext[i];
    if (e.len < a.gran) continue;
    uint64_t start = (e.off + e.len - a.gran) / a.gran * a.gran;
    if (start < e.off) continue;
    if (!arena_carve(i, start, a.gran)) return false;
    *off = start;
    return true;
  }
  return false;
}

void arena_free(uint64_t off) {
  Arena& a = g_arena;
  uint64_t len = 0;
  if (!live_take(off, &len)) return;
  a.used -= len;
  ext_insert(off, len);
  ipc_forget_block(off);
  pthread_cond_broadcast(&a.cv);
}

bool arena_live_find(uint64_t off, uint64_t* start, uint64_t* len) {
  Arena& a = g_arena;
  int i = live_lower(off + 1) - 1;  // the last block starting at or before off
  if (i < 0 || off >= a.live[i].off + a.live[i].len) return false;
  *start = a.live[i].off;
  *len = a.live[i].len;
  return true;
}

void arena_room_changed() { pthread_cond_broadcast(&g_arena.cv); }

// owed granules that have arrived (poll without waiting); g_arena.mu held
bool arena_more_locked(int wait_ms) {
  Arena& a = g_arena;
  if (a.reading || a.n >= a.total || a.sock < 0) return false;
  a.reading = true;
  bool r = more_locked_inner(wait_ms);
  a.reading = false;
  if (r) pthread_cond_broadcast(&a.cv);
  return r;
}

// An allocation of `need` bytes found no room while the grant has granules still owed that would
// make room: wait for them (GPUSHARE_HBM_MORE_WAIT_S, default 60 s; the broker ends the stream at
// its --wait-s). One thread polls the socket with g_arena.mu dropped, so frees and allocations
// that fit go on meanwhile; the others wait for it on the condition variable. true: the arena may
// have room now (the caller tries again); false: no owed granule will come.
bool arena_wait_more(uint64_t need) {
  Arena& a = g_arena;
  if (a.n >= a.total || a.sock < 0 || need > a.size - a.used) return false;
  static double limit_s = -1;
  if (limit_s < 0) {
    const char* w = getenv("GPUSHARE_HBM_MORE_WAIT_S");
    limit_s = w ? atof(w) : 60.0;
  }
  if (a.reading) {  // another thread polls: wait for what it receives (or for a free)
    timespec until;
    clock_gettime(CLOCK_REALTIME, &until);
    until.tv_nsec += 100 * 1000 * 1000;
    if (until.tv_nsec >= 1000000000) {
      until.tv_sec += 1;
      until.tv_nsec -= 1000000000;
    }
    pthread_cond_timedwait(&a.cv, &a.mu, &until);
    return true;
  }
  ++g_more_waits;
  uint64_t deadline = mono_ns() + uint64_t(limit_s * 1e9);
  int sock = a.sock;
  while (a.n < a.total && a.sock == sock) {
    a.reading = true;
    pthread_mutex_unlock(&a.mu);
    pollfd p{sock, POLLIN, 0};
    uint64_t t0 = mono_ns();
    int r = poll(&p, 1, 100);
    pthread_mutex_lock(&a.mu);
    g_more_wait_ns += mono_ns() - t0;
    bool grew = r > 0 && more_locked_inner(0);
    a.reading = false;
    pthread_cond_broadcast(&a.cv);
    if (grew) return true;
    if (a.state.load() != 1 || a.sock != sock) return false;
    if (need <= a.size - a.used && arena_fits(need)) return true;  // a free made room meanwhile
    if (mono_ns() > deadline) {
      logf(1, "hbm broker: %d granules still owed after %.0f s: ending the stream", a.total - a.n, limit_s);
      arena_stream_end("timeout");
      return false;
    }
  }
  return false;
}

// Granules beyond the grant for an allocation of `need` bytes the arena cannot hold: "EXTEND k"
// (the broker lends what no grant claims, up to the pod's limit), charged first and mapped after
// the granules there. g_arena.mu held; true if the arena grew.
bool arena_extend_locked(uint64_t need) {
  Arena& a = g_arena;
  if (a.sock < 0 || a.ended || a.reading || a.n < a.total || a.total >= a.limit) return false;
  uint64_t short_by = tail_shortfall(need);
  int k = int((short_by + a.gran - 1) / a.gran);
  if (k < 1) k = 1;
  k = k < a.limit - a.total ? k : a.limit - a.total;
  k = k < kArenaMaxGranules - a.total ? k : kArenaMaxGranules - a.total;
  if (a.charged) {
    uint64_t left = quota_left() / a.gran;
    if (uint64_t(k) > left) k = int(left);
  }
  if (k <= 0) return false;
  if (a.charged && !charge(uint64_t(k) * a.gran)) return false;
  a.reading = true;
  char line[128];
  int n = snprintf(line, sizeof line, "EXTEND %d\n", k);
  int j = -1;
  unsigned long long gj = 0, gg = 0;
  if (send(a.sock, line, size_t(n), MSG_NOSIGNAL) == n) {
    for (;;) {
      if (!recv_line_ms(a.sock, line, sizeof line, 2000)) break;
      if (broker_notice(line)) continue;
      if (sscanf(line, "XFDS %llu %llu", &gj, &gg) == 2 && gg == a.gran && gj <= (unsigned long long)k) j = int(gj);
      break;
    }
  }
  int fds[kArenaMaxGranules];
  bool ok = j > 0 && recv_fds(a.sock, fds, j);
  if (j < 0) {  // no answer (an older broker, or it went away): ask no more
    a.ended = true;
    logf(1, "hbm broker: no answer to EXTEND (%s): the rest of the quota comes from the driver", line);
  }
  if (ok) {
    char* at = a.base + uint64_t(a.n) * a.gran;
    int failed = import_and_map(fds, j, a.h + a.n, at, a.gran, a.by_address);
    if (failed || !set_rw(at, uint64_t(j) * a.gran, g_dev)) {
      auto un = real_hipMemUnmap();
      auto rel = real_hipMemRelease();
      Depth d;
      for (int i = 0; i < j; ++i) {
        if (a.h[a.n + i]) {
          if (un) (void)un(at + uint64_t(i) * a.gran, a.gran);
          if (rel) (void)rel(a.h[a.n + i]);
          a.h[a.n + i] = nullptr;
        }
        close(fds[i]);
      }
      ok = false;
      a.ended = true;  // the broker counts them as ours until the connection ends: ask no more
    }
  }
  a.reading = false;
  if (!ok) {
    if (a.charged) uncharge(uint64_t(k) * a.gran);
    return false;
  }
  for (int i = 0; i < j; ++i) a.fd[a.n + i] = fds[i];
  ext_insert(uint64_t(a.n) * a.gran, uint64_t(j) * a.gran);
  a.n += j;
  a.total += j;
  a.extra += j;
  a.size += uint64_t(j) * a.gran;
  if (a.charged && j < k) uncharge(uint64_t(k - j) * a.gran);
  ++g_extends;
  g_extended += uint64_t(j);
  logf(1, "hbm broker: %d granules beyond the grant (%d of %d, limit %d)", j, a.n, a.total, a.limit);
  pthread_cond_broadcast(&a.cv);
  return true;
}

// what EXTEND could lend now, in granules (-1: not asked: the stream is not complete, or the
// socket is busy); g_arena.mu held
int arena_avail_locked() {
  Arena& a = g_arena;
  if (a.sock < 0 || a.ended || a.reading || a.n < a.total) return -1;
  if (a.total >= a.limit) return 0;
  a.reading = true;
  char line[128];
  int r = -1;
  if (send(a.sock, "AVAIL\n", 6, MSG_NOSIGNAL) == 6) {
    for (;;) {
      if (!recv_line_ms(a.sock, line, sizeof line, 500)) break;
      if (broker_notice(line)) continue;
      if (sscanf(line, "AVAIL %d", &r) != 1) r = -1;
      break;
    }
  }
  if (r < 0) a.ended = true;  // an older broker: no beyond-grant lending
  a.reading = false;
  int room = a.limit - a.total;
  return r < 0 ? 0 : (r < room ? r : room);
}

// 1: served from the arena (*e set), 0: not the arena's (pass through to the driver)
int arena_try_alloc(void** ptr, size_t size, hipError_t* e) {
  if (!arena_configured() || size == 0 || t_depth) return 0;
  Arena& a = g_arena;
  pthread_mutex_lock(&a.mu);
  if (a.state == 0) arena_take();
  if (a.state != 1) {
    pthread_mutex_unlock(&a.mu);
    return 0;
  }
  if (frees_pending()) reap_frees(false);
  while (a.n < a.total && arena_more_locked(0)) {
  }  // owed granules that have arrived
  bool ok = arena_alloc(size, ptr);
  if (!ok && frees_pending()) {  // room that deferred frees will give back: wait for them
    reap_frees(true);
    ok = arena_alloc(size, ptr);
  }
  while (!ok && arena_wait_more(size)) ok = arena_alloc(size, ptr);  // room the broker still owes
  if (!ok && arena_extend_locked(size)) ok = arena_alloc(size, ptr);  // granules beyond the grant
  if (!ok) {
    ++g_driver_allocs;
    g_driver_bytes += size;
  }
  pthread_mutex_unlock(&a.mu);
  if (!ok) {
    logf(1, "hbm broker arena: %zu bytes from the driver (arena used %llu of %llu)", size,
         (unsigned long long)a.used, (unsigned long long)a.size);
    return 0;
  }
  *e = hipSuccess;
  return 1;
}

}  // namespace gs

using namespace gs;

// Hand the arena back to the broker now (the pod is retiring and freed everything). Returns 1 if
// released, 0 if there is no arena, -1 if allocations are still live in it.
// The fast exit on demand, for a process about to end (probes): every queue destroyed, every
// noted import (and, with GPUSHARE_SHIM_FREE_ALLOCS_AT_EXIT=1, every KFD allocation) freed. The
// process must not touch the GPU afterwards.
GS_EXPORT int gpushare_shim_fast_exit_release() {
  fast_release("api");
  return 0;
}

GS_EXPORT int gpushare_shim_arena_release() {
  Arena& a = g_arena;
  pthread_mutex_lock(&a.mu);
  if (a.state != 1) {
    pthread_mutex_unlock(&a.mu);
    return 0;
  }
  if (frees_pending()) reap_frees(true);
  if (a.nlive || a.reading) {  // (granules lent to VMM windows are live blocks too)
    pthread_mutex_unlock(&a.mu);
    return -1;
  }
  arena_unmap_locked();
  if (a.rt_version > 0 && a.rt_version < 70100000 && env_u64("GPUSHARE_HBM_FREE_KEPT", 1)) {
    // HIP 7.0 keeps the KFD imports of the released handles: free them, so the broker sees its
    // granules' references gone now rather than at this process's teardown
    uint64_t t = mono_ns();
    int n = imports_free(kArenaImportTag);
    g_rel_ns[4] = mono_ns() - t;
    logf(1, "hbm broker: freed %d KFD imports the runtime kept", n);
  }
  if (a.charged) uncharge(a.size);
  a.charged = false;
  close(a.sock);
  a.sock = -1;
  a.state.store(-1, std::memory_order_release);
  pthread_mutex_unlock(&a.mu);
  return 1;
}

GS_EXPORT int gpushare_shim_arena_release_timing(uint64_t* sync_ns, uint64_t* unmap_ns, uint64_t* addr_free_ns,
                                                 uint64_t* release_ns, uint64_t* kfd_free_ns) {
  pthread_mutex_lock(&g_arena.mu);
  *sync_ns = g_rel_ns[0];
  *unmap_ns = g_rel_ns[1];
  *addr_free_ns = g_rel_ns[2];
  *release_ns = g_rel_ns[3];
  *kfd_free_ns = g_rel_ns[4];
  pthread_mutex_unlock(&g_arena.mu);
  return 1;
}

// where the arena's TAKE spent its time (ns): connect, the broker's answer (a grant not there
// yet, granules still held by a retiring pod), import + map; 0 when there is no arena
GS_EXPORT int gpushare_shim_arena_timing(uint64_t* connect_ns, uint64_t* wait_ns, uint64_t* map_ns) {
  int on = g_arena.state.load(std::memory_order_acquire) == 1;
  if (connect_ns) *connect_ns = g_take_connect_ns;
  if (wait_ns) *wait_ns = g_take_wait_ns;
  if (map_ns) *map_ns = g_take_map_ns;
  return on;
}

// a streaming TAKE after it returned: allocations that waited for owed granules (count, ns), the
// MORE batches received and the ns spent importing + mapping them, granules mapped and granted;
// of the TAKE's first batch: its granules, and the ns of its address reservation and access
GS_EXPORT int gpushare_shim_arena_stream(uint64_t* waits, uint64_t* wait_ns, uint64_t* msgs, uint64_t* map_ns,
                                         uint64_t* mapped, uint64_t* granted, uint64_t* first, uint64_t* reserve_ns,
                                         uint64_t* access_ns) {
  Arena& a = g_arena;
  pthread_mutex_lock(&a.mu);
  int on = a.state == 1;
  if (waits) *waits = g_more_waits;
  if (wait_ns) *wait_ns = g_more_wait_ns;
  if (msgs) *msgs = g_more_msgs;
  if (map_ns) *map_ns = g_more_map_ns;
  if (mapped) *mapped = on ? uint64_t(a.n) : 0;
  if (granted) *granted = on ? uint64_t(a.total) : 0;
  if (first) *first = g_take_first;
  if (reserve_ns) *reserve_ns = g_take_reserve_ns;
  if (access_ns) *access_ns = g_take_access_ns;
  pthread_mutex_unlock(&a.mu);
  return on;
}

// beyond the grant: EXTEND requests that got granules and the granules they got; allocations
// the arena could not serve (the driver's, charged to the ledger) and their bytes; the limit
GS_EXPORT int gpushare_shim_arena_extra(uint64_t* extends, uint64_t* extended, uint64_t* driver_allocs,
                                        uint64_t* driver_bytes, uint64_t* limit) {
  Arena& a = g_arena;
  pthread_mutex_lock(&a.mu);
  int on = a.state == 1;
  if (extends) *extends = g_extends;
  if (extended) *extended = g_extended;
  if (driver_allocs) *driver_allocs = g_driver_allocs;
  if (driver_bytes) *driver_bytes = g_driver_bytes;
  if (limit) *limit = on ? uint64_t(a.limit) : 0;
  pthread_mutex_unlock(&a.mu);
  return on;
}

// the process's first granule import and map (ns): the runtime's one-time work inside the TAKE;
// and how long the TAKE waited for the broker's answer line
GS_EXPORT int gpushare_shim_arena_first(uint64_t* import_ns, uint64_t* map_ns, uint64_t* header_ns) {
  if (import_ns) *import_ns = g_first_import_ns;
  if (map_ns) *map_ns = g_first_map_ns;
  if (header_ns) *header_ns = g_take_header_ns;
  return g_first_import_ns != 0;
}

// (size, used) of the arena; 0 when there is none
// the arena's address (0 without one): tests and tools check its alignment
GS_EXPORT uint64_t gpushare_shim_arena_base() { return reinterpret_cast<uint64_t>(g_arena.base); }

GS_EXPORT int gpushare_shim_arena_stats(uint64_t* size, uint64_t* used) {
  Arena& a = g_arena;
  pthread_mutex_lock(&a.mu);
  int on = a.state == 1;
  if (on && frees_pending()) reap_frees(false);  // frees whose streams are past them are not in use
  if (size) *size = on ? a.size : 0;
  if (used) *used = on ? a.used : 0;
  pthread_mutex_unlock(&a.mu);
  return on;
}
