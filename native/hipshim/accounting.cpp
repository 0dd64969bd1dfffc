// libgpushare_hipquota.so — per-container HBM quota for GPU programs (LD_PRELOAD interposer).
//
// The reference plugin only *describes* a container's GPU-memory share through env vars
// (ALIYUN_COM_GPU_MEM_CONTAINER / _DEV, allocate.go:114-129) and relies on Alibaba's closed
// cGPU kernel module to enforce it (CGPU_DISABLE switches it off, allocate.go:125-127).
// On MI355X the plugin mounts this library into every shared container and preloads it:
//
//   quota = GPUSHARE_QUOTA_BYTES                      (the plugin sets it: HBM bytes * CONTAINER / DEV)
//           else real_HBM_bytes * CONTAINER / DEV     (HBM bytes from the KFD topology / HIP)
//
// Enforcement point (default, GPUSHARE_SHIM_MODE=kfd): the KFD boundary (kfd.cpp). Every byte of
// HBM a process owns is created by one ioctl on /dev/kfd — AMDKFD_IOC_ALLOC_MEMORY_OF_GPU with the
// VRAM flag — issued by ROCr (libhsa-runtime64 imports ioctl from libc through its PLT, so a
// preloaded ioctl sees it) and released by AMDKFD_IOC_FREE_MEMORY_OF_GPU. Charging there covers
// what the HIP entry points cannot see: hipMallocAsync pools that keep memory after hipFreeAsync,
// hipMallocArray / 3D arrays, scratch (private segment) buffers, code objects, queue and staging
// buffers allocated inside the runtime, and programs that call HSA directly. Over quota the ioctl
// fails with ENOMEM, exactly as when HBM runs out: ROCr trims its caches and retries, then reports
// HSA_STATUS_ERROR_OUT_OF_RESOURCES / hipErrorOutOfMemory.
//
// hipMemGetInfo / hipDeviceTotalMem / hipGetDeviceProperties are also interposed (api.cpp) so
// frameworks see the quota as the device total and what the pod can still obtain as free memory.
//
// GPUSHARE_SHIM_MODE=hip keeps the older HIP-API accounting (hipMalloc family + VMM, charges
// rounded to the 2 MiB CDNA4 fragment, GPUSHARE_ALLOC_GRANULE) for runtimes whose KFD traffic
// is not visible; the two modes never both charge.
//
// All processes of one container share one ledger in POSIX shared memory (GPUSHARE_LEDGER) or
// a file in a host directory (GPUSHARE_LEDGER_DIR): a global atomic total plus one slot per
// process, so a crashed process's charge is reclaimed by the next allocation that needs room.
// A forked child starts with an empty allocation table and its own slot (a child does not
// inherit its parent's KFD allocations).
//
// This unit holds the ledger, the allocation table, initialisation and symbol resolution. The
// other units are listed in shim.h, with the lock order.
//
// Limits (documented, by construction): enforcement is cooperative — a process that drops
// LD_PRELOAD or issues the ioctl through a raw syscall is not charged. Memory imported from
// another process (dma-buf / IPC) is charged to its exporter only. KFD allocations issued
// while the shim itself is initialising (the runtime's own start-up, reached from init) pass
// uncharged. The node's quota watchdog (amdgpu fdinfo / VRAM usage, quota/watchdog.py) is the
// backstop for what the shim cannot see.
//
// The library does not link libamdhip64 or libhsa-runtime64: the real entry points are
// resolved at run time from whichever runtime the process loaded (PyTorch ships its own copy).
// It is linked with -static-libstdc++ -static-libgcc so it loads into any tenant image.
#include "shim.h"

#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <link.h>
#include <signal.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/sysmacros.h>
#include <time.h>
#include <unistd.h>

namespace gs {

State g;
std::atomic<bool> g_initializing{false};
std::atomic<bool> g_released{false};
thread_local int t_depth = 0;

namespace {
pthread_once_t g_once = PTHREAD_ONCE_INIT;
std::atomic<int> g_env_mode{-1};  // GPUSHARE_SHIM_MODE read without initialising
}  // namespace

void logf(int level, const char* fmt, ...) {
  if (g.log < level) return;
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  fprintf(stderr, "[gpushare-hipquota %d] %s\n", (int)getpid(), buf);
}

uint64_t mono_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return uint64_t(t.tv_sec) * 1000000000ull + uint64_t(t.tv_nsec);
}

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  unsigned long long x = strtoull(v, &end, 10);
  return (end && end != v) ? (uint64_t)x : dflt;
}

// ---- real symbol resolution ---------------------------------------------------------------
namespace {
void* g_hip_handle = nullptr;

int find_hip_cb(struct dl_phdr_info* info, size_t, void* data) {
  if (info->dlpi_name && strstr(info->dlpi_name, "libamdhip64.so")) {
    *static_cast<const char**>(data) = info->dlpi_name;
    return 1;
  }
  return 0;
}
}  // namespace

void* resolve(const char* name) {
  void* p = dlsym(RTLD_NEXT, name);
  if (p) return p;
  if (!g_hip_handle) {
    const char* path = nullptr;
    dl_iterate_phdr(find_hip_cb, &path);
    if (path) g_hip_handle = dlopen(path, RTLD_NOLOAD | RTLD_LAZY);
    if (!g_hip_handle) g_hip_handle = dlopen("libamdhip64.so.7", RTLD_LAZY | RTLD_GLOBAL);
    if (!g_hip_handle) g_hip_handle = dlopen("libamdhip64.so", RTLD_LAZY | RTLD_GLOBAL);
  }
  return g_hip_handle ? dlsym(g_hip_handle, name) : nullptr;
}

#define GS_DEF_REAL(ret, name, ...)                                            \
  name##_t real_##name() {                                                     \
    static std::atomic<name##_t> fn{nullptr};                                  \
    name##_t f = fn.load(std::memory_order_acquire);                           \
    if (!f) {                                                                  \
      f = reinterpret_cast<name##_t>(resolve(#name));                          \
      fn.store(f, std::memory_order_release);                                  \
    }                                                                          \
    return f;                                                                  \
  }
GS_REAL_FUNCS(GS_DEF_REAL)
#undef GS_DEF_REAL

namespace {
std::atomic<ioctl_t> g_real_ioctl{nullptr};
}

ioctl_t real_ioctl() {
  ioctl_t f = g_real_ioctl.load(std::memory_order_acquire);
  if (!f) {
    f = reinterpret_cast<ioctl_t>(dlsym(RTLD_NEXT, "ioctl"));
    g_real_ioctl.store(f, std::memory_order_release);
  }
  return f;
}

// ---- allocation table (sharded): pointer (hip mode) or KFD handle (kfd mode) -> charge -------
// No libstdc++ containers: the shim must not pull libstdc++'s runtime (exception objects need a
// newer glibc than tenant images may have). Open addressing, linear probing, key 0 = empty,
// key ~0 = deleted; grows at 50 % load.
Shard g_shards[64];

namespace {
Shard& shard_of(uint64_t k) { return g_shards[((k >> 21) ^ k) & 63]; }

size_t slot_of(uint64_t k, size_t cap) { return (size_t)((k * 0x9E3779B97F4A7C15ull) >> 20) & (cap - 1); }

bool grow(Shard& s) {
  size_t ncap = s.cap ? s.cap * 2 : 64;
  auto* nk = static_cast<uint64_t*>(calloc(ncap, sizeof(uint64_t)));
  auto* nv = static_cast<uint64_t*>(calloc(ncap, sizeof(uint64_t)));
  if (!nk || !nv) {
    free(nk);
    free(nv);
    return false;
  }
  size_t live = 0;
  for (size_t i = 0; i < s.cap; ++i) {
    uint64_t k = s.keys[i];
    if (k == kEmpty || k == kDeleted) continue;
    size_t j = slot_of(k, ncap);
    while (nk[j] != kEmpty) j = (j + 1) & (ncap - 1);
    nk[j] = k;
    nv[j] = s.vals[i];
    ++live;
  }
  free(s.keys);
  free(s.vals);
  s.keys = nk;
  s.vals = nv;
  s.cap = ncap;
  s.used = live;
  return true;
}
}  // namespace

void track(uint64_t k, uint64_t charge) {
  if (k == kEmpty || k == kDeleted) return;
  Shard& s = shard_of(k);
  pthread_mutex_lock(&s.mu);
  if ((s.used + 1) * 2 > s.cap && !grow(s)) {
    pthread_mutex_unlock(&s.mu);
    return;  // out of host memory: the charge stays (conservative)
  }
  size_t i = slot_of(k, s.cap), tomb = (size_t)-1;
  for (;; i = (i + 1) & (s.cap - 1)) {
    if (s.keys[i] == k) {
      s.vals[i] = charge;
      break;
    }
    if (s.keys[i] == kDeleted && tomb == (size_t)-1) tomb = i;
    if (s.keys[i] == kEmpty) {
      if (tomb != (size_t)-1) {
        i = tomb;
      } else {
        ++s.used;
      }
      s.keys[i] = k;
      s.vals[i] = charge;
      break;
    }
  }
  pthread_mutex_unlock(&s.mu);
}

uint64_t untrack(uint64_t k) {
  if (k == kEmpty || k == kDeleted) return 0;
  Shard& s = shard_of(k);
  pthread_mutex_lock(&s.mu);
  uint64_t c = 0;
  if (s.cap) {
    for (size_t i = slot_of(k, s.cap), n = 0; n < s.cap; i = (i + 1) & (s.cap - 1), ++n) {
      if (s.keys[i] == kEmpty) break;
      if (s.keys[i] == k) {
        c = s.vals[i];
        s.keys[i] = kDeleted;
        break;
      }
    }
  }
  pthread_mutex_unlock(&s.mu);
  return c;
}

// ---- ledger --------------------------------------------------------------------------------
namespace {
bool pid_alive(int32_t pid) { return pid > 0 && (kill(pid, 0) == 0 || errno != ESRCH); }

void reclaim_slot(LedgerShm* L, int i, int32_t dead_pid) {
  Slot& s = L->slots[i];
  int32_t expect = dead_pid;
  if (!s.pid.compare_exchange_strong(expect, -1)) return;  // someone else reclaims it
  uint64_t u = s.used.exchange(0);
  L->total.fetch_sub(u);
  s.pid.store(0);
  logf(1, "reclaimed %llu bytes from dead pid %d", (unsigned long long)u, dead_pid);
}

int acquire_slot(LedgerShm* L) {
  int32_t me = getpid();
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = 0; i < kSlots; ++i) {
      int32_t expect = 0;
      if (L->slots[i].pid.compare_exchange_strong(expect, me)) {
        L->slots[i].used.store(0);
        return i;
      }
    }
    reclaim_dead(L);
  }
  return -1;
}

// GPUSHARE_SHIM_DIAG=1: before each charge, check that the ledger page is still mapped; if it
// is not, print the process's mappings around it and abort (field diagnosis of a lost ledger).
void diag_check(LedgerShm* L) {
  unsigned char v;
  void* page = reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(L) & ~uintptr_t(4095));
  if (mincore(page, 4096, &v) == 0 || errno != ENOMEM) return;
  fprintf(stderr, "[gpushare-hipquota %d] ledger %p (%s) is no longer mapped\n", (int)getpid(), (void*)L,
          g.ledger_name);
  FILE* f = fopen("/proc/self/maps", "re");
  if (f) {
    char ln[512];
    uintptr_t a = reinterpret_cast<uintptr_t>(L);
    while (fgets(ln, sizeof ln, f)) {
      unsigned long lo = 0, hi = 0;
      if (sscanf(ln, "%lx-%lx", &lo, &hi) == 2 && hi + (64ul << 20) > a && lo < a + (64ul << 20)) fputs(ln, stderr);
    }
    fclose(f);
  }
  abort();
}
}  // namespace

int reclaim_dead(LedgerShm* L) {
  int n = 0;
  for (int i = 0; i < kSlots; ++i) {
    int32_t p = L->slots[i].pid.load();
    if (p > 0 && p != getpid() && !pid_alive(p)) {
      reclaim_slot(L, i, p);
      ++n;
    }
  }
  return n;
}

bool charge(uint64_t bytes) {
  if (g_released.load(std::memory_order_relaxed)) return true;  // process teardown
  LedgerShm* L = g.ledger;
  if (g.diag) diag_check(L);
  uint64_t quota = g.quota.load(std::memory_order_relaxed);
  bool reclaimed = false, gced = false;
  uint64_t cur = L->total.load();
  for (;;) {
    if (quota && cur + bytes > quota) {
      if (!reclaimed && reclaim_dead(L) > 0) {
        reclaimed = true;
        cur = L->total.load();
        continue;
      }
      if (!gced) {  // GEM files that were still referred to when their fd closed may be gone now
        gced = true;
        if (linger_gc() > 0) {
          cur = L->total.load();
          continue;
        }
      }
      L->denied.fetch_add(1);
      return false;
    }
    if (L->total.compare_exchange_weak(cur, cur + bytes)) break;
  }
  if (g.slot >= 0) L->slots[g.slot].used.fetch_add(bytes);
  uint64_t now = cur + bytes, pk = L->peak.load();
  while (now > pk && !L->peak.compare_exchange_weak(pk, now)) {
  }
  return true;
}

void uncharge(uint64_t bytes) {
  if (!bytes || g_released.load(std::memory_order_relaxed)) return;
  if (g.slot >= 0) g.ledger->slots[g.slot].used.fetch_sub(bytes);
  g.ledger->total.fetch_sub(bytes);
}

uint64_t quota_left() {
  if (!enabled()) return 0;
  uint64_t quota = g.quota.load(), used = g.ledger->total.load();
  return quota && used < quota ? quota - used : 0;
}

uint64_t round_up(uint64_t n, uint64_t g_) { return g_ ? (n + g_ - 1) / g_ * g_ : n; }
uint64_t charge_of(size_t n) { return n == 0 ? 0 : round_up((uint64_t)n, g.granule); }

hipError_t deny(size_t n) {
  logf(1, "deny %zu bytes: used %llu of %llu", n, (unsigned long long)g.ledger->total.load(),
       (unsigned long long)g.quota.load());
  return hipErrorOutOfMemory;
}

// HBM bytes of the GPU whose KFD gpu_id is `gpu_id`, from the KFD topology (no HIP call: this
// runs inside ROCr's own initialisation). 0 when unknown.
uint64_t kfd_vram_bytes(uint32_t gpu_id) {
  char base[256];  // GPUSHARE_KFD_SYSFS: root prefix of a synthetic topology (tests)
  const char* root = getenv("GPUSHARE_KFD_SYSFS");
  snprintf(base, sizeof base, "%s/sys/class/kfd/kfd/topology/nodes", root ? root : "");
  DIR* d = opendir(base);
  if (!d) return 0;
  uint64_t out = 0;
  while (struct dirent* e = readdir(d)) {
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    char path[256], buf[64];
    snprintf(path, sizeof path, "%s/%s/gpu_id", base, e->d_name);
    FILE* f = fopen(path, "re");
    if (!f) continue;
    unsigned long id = 0;
    bool ok = fgets(buf, sizeof buf, f) && sscanf(buf, "%lu", &id) == 1;
    fclose(f);
    if (!ok || id != gpu_id) continue;
    for (int bank = 0; bank < 16 && !out; ++bank) {
      snprintf(path, sizeof path, "%s/%s/mem_banks/%d/properties", base, e->d_name, bank);
      FILE* p = fopen(path, "re");
      if (!p) break;
      char line[128];
      unsigned long long heap = 0, size = 0;
      while (fgets(line, sizeof line, p)) {
        sscanf(line, "heap_type %llu", &heap);
        sscanf(line, "size_in_bytes %llu", &size);
      }
      fclose(p);
      if (heap == 1 || heap == 2) out = size;  // HSA_HEAPTYPE_FRAME_BUFFER_PUBLIC / _PRIVATE
    }
    break;
  }
  closedir(d);
  return out;
}

// HBM bytes of the GPU behind render-node fd ``fd`` (amdgpu sysfs), 0 when unknown.
uint64_t render_vram_bytes(int fd) {
  struct stat st;   // raw syscall: glibc's fstat is versioned GLIBC_2.33, newer than tenant images'
  if (syscall(SYS_fstat, fd, &st) != 0 || !S_ISCHR(st.st_mode)) return 0;
  char path[256], buf[64];
  const char* root = getenv("GPUSHARE_KFD_SYSFS");
  snprintf(path, sizeof path, "%s/sys/dev/char/%u:%u/device/mem_info_vram_total", root ? root : "",
           (unsigned)major(st.st_rdev), (unsigned)minor(st.st_rdev));
  FILE* f = fopen(path, "re");
  if (!f) return 0;
  unsigned long long v = 0;
  if (!fgets(buf, sizeof buf, f) || sscanf(buf, "%llu", &v) != 1) v = 0;
  fclose(f);
  return v;
}

void set_quota_from_device_bytes(uint64_t tot) {
  if (!tot || !g.ctr || !g.dev) return;
  uint64_t q = (uint64_t)((__uint128_t)tot * g.ctr / g.dev);
  if (q > tot) q = tot;
  uint64_t zero = 0;
  if (g.ledger->quota.compare_exchange_strong(zero, q)) logf(1, "quota %llu bytes from %llu device bytes",
                                                            (unsigned long long)q, (unsigned long long)tot);
  g.quota.store(g.ledger->quota.load());
}

namespace {
// atexit: hand the slot back. The runtime's own teardown (later destructors) still frees its
// allocations through the ioctl; from here on the ledger is no longer this process's to touch.
void release_slot_at_exit() {
  if (!g.enabled || !g.ledger || g.slot < 0) return;
  g_released.store(true);
  Slot& s = g.ledger->slots[g.slot];
  uint64_t u = s.used.exchange(0);
  g.ledger->total.fetch_sub(u);
  s.pid.store(0);
  g.slot = -1;
}

void atfork_child() {
  if (!g.enabled || !g.ledger) return;
  // The child is a new process: it owns none of the parent's allocations (KFD allocations are
  // per process; the parent's pointers are the parent's to free) and gets its own slot.
  for (auto& s : g_shards) {
    pthread_mutex_init(&s.mu, nullptr);  // a lock held by another parent thread at fork time is void here
    if (s.cap) memset(s.keys, 0, s.cap * sizeof(uint64_t));
    s.used = 0;
  }
  if (g.ledger == &g.local) {  // a process-private ledger: the copy still holds the parent's charges
    g.local.total.store(0);
    g.local.peak.store(0);
    for (auto& sl : g.local.slots) {
      sl.pid.store(0);
      sl.used.store(0);
    }
  }
  g.slot = acquire_slot(g.ledger);
}

// Address range for the ledger, reserved when the library loads — before the runtime (or
// anything else) starts mapping and unmapping — so no one else can believe it is theirs.
constexpr size_t kLedgerMapBytes = (sizeof(LedgerShm) + 4095) & ~size_t(4095);
void* g_ledger_va = nullptr;

__attribute__((constructor)) void reserve_ledger_va() {
  void* p = mmap(nullptr, kLedgerMapBytes, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (p != MAP_FAILED) g_ledger_va = p;
}

// Room in the process's fd table for a broker arena's granule fds, made while the process is
// still single-threaded. The kernel grows an fd table that is full; in a multi-threaded process
// (a pod whose HIP runtime is up) each growth waits for an RCU grace period. Measured on MI355X:
// receiving 60-120 granule fds at a TAKE took 115-210 ms, 30 (no growth) 0.014 ms. A table
// grown here, at load time, never needs to grow for the arena. GPUSHARE_SHIM_FD_RESERVE=0 skips it.
// A forked child gets a table only as large as its highest open fd, so the child grows it again
// right after the fork, while it is still single-threaded.
void grow_fd_table() {
  rlimit rl;
  if (getrlimit(RLIMIT_NOFILE, &rl) != 0 || rl.rlim_cur < 256) return;
  long top = long(rl.rlim_cur > 2048 ? 2048 : rl.rlim_cur) - 1;
  if (fcntl(int(top), F_GETFD) != -1) return;  // in use: the table is that large already
  long d = syscall(SYS_openat, AT_FDCWD, "/dev/null", O_RDONLY | O_CLOEXEC);
  if (d < 0) return;
  if (syscall(SYS_dup3, d, top, O_CLOEXEC) == top) syscall(SYS_close, top);
  syscall(SYS_close, d);
}

__attribute__((constructor)) void reserve_fd_table() {
  const char* v = getenv("GPUSHARE_SHIM_FD_RESERVE");
  if (v && !strcmp(v, "0")) return;
  grow_fd_table();
  pthread_atfork(nullptr, nullptr, grow_fd_table);
}

void init_body() {
  g.log = (int)env_u64("GPUSHARE_SHIM_LOG", 0);
  g.diag = (int)env_u64("GPUSHARE_SHIM_DIAG", 0);
  const char* dis = getenv("CGPU_DISABLE");
  if (dis && !strcmp(dis, "true")) {
    logf(1, "CGPU_DISABLE=true: quota enforcement off");
    return;
  }
  const char* mode = getenv("GPUSHARE_SHIM_MODE");
  g.mode = (mode && !strcmp(mode, "hip")) ? kModeHip : kModeKfd;
  g.granule = g.mode == kModeHip ? env_u64("GPUSHARE_ALLOC_GRANULE", kDefaultGranule) : 1;
  uint64_t q = env_u64("GPUSHARE_QUOTA_BYTES", 0);
  g.ctr = env_u64("ALIYUN_COM_GPU_MEM_CONTAINER", 0);
  g.dev = env_u64("ALIYUN_COM_GPU_MEM_DEV", 0);
  if (!q && (!g.ctr || !g.dev)) {
    logf(1, "no quota configured: pass-through");
    return;
  }
  if (!q && g.mode == kModeHip) {
    size_t fr = 0, tot = 0;
    t_depth++;
    hipError_t e = real_hipMemGetInfo() ? real_hipMemGetInfo()(&fr, &tot) : hipErrorNotInitialized;
    t_depth--;
    if (e != hipSuccess || tot == 0) {
      logf(0, "cannot read device memory (err %d): pass-through", (int)e);
      return;
    }
    q = (uint64_t)((__uint128_t)tot * g.ctr / g.dev);
    if (q > tot) q = tot;
  }
  // kfd mode without GPUSHARE_QUOTA_BYTES: the quota is derived at the first VRAM allocation
  // from that GPU's HBM size (KFD topology), see kfd_alloc().
  const char* ln = getenv("GPUSHARE_LEDGER");
  if (ln && *ln) {
    snprintf(g.ledger_name, sizeof g.ledger_name, "%s%s", ln[0] == '/' ? "" : "/", ln);
    // GPUSHARE_LEDGER_DIR: file-backed ledger in a directory the plugin mounts from the host,
    // so the node agent can read every container's usage / peak / denials (a container's
    // /dev/shm is private to its pod); otherwise a POSIX shm object.
    const char* dir = getenv("GPUSHARE_LEDGER_DIR");
    int fd = -1;
    if (dir && *dir) {
      char path[512];
      snprintf(path, sizeof path, "%s%s.ledger", dir, g.ledger_name);
      fd = open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0644);
      if (fd >= 0) snprintf(g.ledger_name, sizeof g.ledger_name, "%s", path);
    } else {
      fd = shm_open(g.ledger_name, O_RDWR | O_CREAT, 0600);
    }
    if (fd >= 0 && ftruncate(fd, sizeof(LedgerShm)) == 0) {
      // Onto the range reserved at load time: this runs inside the runtime's first VRAM ioctl,
      // and ROCr maps ranges it probed free just before that ioctl MAP_FIXED right after it —
      // a fresh mapping placed there would be replaced under us (measured on MI355X).
      void* p = g_ledger_va ? mmap(g_ledger_va, sizeof(LedgerShm), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fd, 0)
                            : mmap(nullptr, sizeof(LedgerShm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (p != MAP_FAILED) {
        g.ledger = static_cast<LedgerShm*>(p);
        uint64_t zero = 0;  // first process initialises; ftruncate zero-fills
        if (g.ledger->magic.compare_exchange_strong(zero, kMagic) && q) g.ledger->quota.store(q);
      }
    }
    if (fd >= 0) close(fd);
    if (!g.ledger) logf(0, "shm ledger %s unavailable (%s): per-process quota", g.ledger_name, strerror(errno));
  }
  if (!g.ledger) {
    g.ledger = &g.local;
    g.local.magic.store(kMagic);
    g.local.quota.store(q);
  }
  if (q) {
    uint64_t zero = 0;
    g.ledger->quota.compare_exchange_strong(zero, q);
  }
  g.quota.store(g.ledger->quota.load());
  g.slot = acquire_slot(g.ledger);
  g.enabled = true;
  atexit(release_slot_at_exit);
  pthread_atfork(nullptr, nullptr, atfork_child);
  if (g.diag) fprintf(stderr, "[gpushare-hipquota %d] ledger %s mapped at %p\n", (int)getpid(), g.ledger_name, (void*)g.ledger);
  logf(1, "mode %s, quota %llu bytes (%.2f GiB%s), ledger %s slot %d", g.mode == kModeKfd ? "kfd" : "hip",
       (unsigned long long)g.quota.load(), (double)g.quota.load() / (1ull << 30),
       g.quota.load() ? "" : ", from the first GPU allocation", g.ledger_name[0] ? g.ledger_name : "(local)",
       g.slot);
}

void init() {
  g_initializing.store(true);
  init_body();
  g_initializing.store(false);
}
}  // namespace

// The accounting mode from the environment, without running init(): the ioctl interposer
// must know whether it charges at all before it may touch the once-control.
int env_mode() {
  int m = g_env_mode.load(std::memory_order_relaxed);
  if (m < 0) {
    const char* v = getenv("GPUSHARE_SHIM_MODE");
    m = (v && !strcmp(v, "hip")) ? kModeHip : kModeKfd;
    g_env_mode.store(m, std::memory_order_relaxed);
  }
  return m;
}

bool enabled() {
  pthread_once(&g_once, init);
  return g.enabled;
}

}  // namespace gs

using namespace gs;

// ---- introspection (tests, metrics) --------------------------------------------------------
GS_EXPORT int gpushare_shim_stats(uint64_t* used, uint64_t* quota, uint64_t* denied, uint64_t* peak) {
  if (!enabled()) return 0;
  reclaim_dead(g.ledger);  // report live processes' usage only
  if (used) *used = g.ledger->total.load();
  if (quota) *quota = g.quota.load();
  if (denied) *denied = g.ledger->denied.load();
  if (peak) *peak = g.ledger->peak.load();
  return 1;
}

GS_EXPORT uint64_t gpushare_shim_granule() { return g.granule; }

// 0 = kfd (ioctl boundary), 1 = hip (HIP-API accounting), -1 = disabled / pass-through.
GS_EXPORT int gpushare_shim_mode() { return enabled() ? g.mode : -1; }
