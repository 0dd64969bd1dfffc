// libgpushare_hipquota.so — per-container HBM quota for HIP programs (LD_PRELOAD interposer).
//
// The reference plugin only *describes* a container's GPU-memory share through env vars
// (ALIYUN_COM_GPU_MEM_CONTAINER / _DEV, allocate.go:114-129) and relies on Alibaba's closed
// cGPU kernel module to enforce it (CGPU_DISABLE switches it off, allocate.go:125-127).
// On MI355X the plugin mounts this library into every shared container and preloads it:
//
//   quota = GPUSHARE_QUOTA_BYTES                      if set, else
//           real_HBM_bytes * CONTAINER / DEV           (unit-agnostic: GiB or MiB mode)
//
// Every HIP device-allocation entry point is interposed: hipMalloc, hipExtMallocWithFlags,
// hipMallocManaged, hipMallocAsync, hipMallocFromPoolAsync, hipMallocPitch, hipMalloc3D and the
// VMM path hipMemCreate/hipMemRelease (PyTorch expandable segments); frees release the charge.
// hipMemGetInfo / hipDeviceTotalMem / hipGetDeviceProperties report the quota as the device
// total so frameworks size their pools to the share rather than the whole GPU.
//
// CDNA4 accounting: MI355X's allocator hands out memory in 2 MiB fragments — a 1-byte
// hipMalloc consumes 2 MiB of HBM and 2 MiB + 1 B consumes 4 MiB (measured with
// hipMemGetInfo deltas on MI355X, see profiles/). Charges are rounded to that granule so the
// quota bounds *physical* HBM, not requested bytes (override: GPUSHARE_ALLOC_GRANULE).
//
// All processes of one container share one ledger in POSIX shared memory (GPUSHARE_LEDGER):
// a global atomic total plus one slot per process, so a crashed process's charge is reclaimed
// by the next allocation that needs room (its pid no longer exists).
//
// The library does not link libamdhip64: the real entry points are resolved at run time from
// whichever HIP runtime the process loaded (PyTorch ships its own copy).

#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <hip/hip_deprecated.h>

#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <link.h>
#include <pthread.h>
#include <signal.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <mutex>
#include <unordered_map>

#undef hipGetDeviceProperties

#define GS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

constexpr uint64_t kMagic = 0x67707573686172ULL;  // "gpushar"
constexpr int kSlots = 256;
constexpr uint64_t kDefaultGranule = 2ull << 20;

struct Slot {
  std::atomic<int32_t> pid;
  int32_t pad;
  std::atomic<uint64_t> used;
};

struct LedgerShm {
  std::atomic<uint64_t> magic;
  std::atomic<uint64_t> quota;
  std::atomic<uint64_t> total;
  std::atomic<uint64_t> denied;
  std::atomic<uint64_t> peak;
  Slot slots[kSlots];
};

struct State {
  bool enabled = false;
  int log = 0;
  uint64_t quota = 0;
  uint64_t granule = kDefaultGranule;
  LedgerShm* ledger = nullptr;
  LedgerShm local{};  // used when no shared ledger is configured
  int slot = -1;
  char ledger_name[128] = {0};
};

State g;
std::once_flag g_once;
thread_local int t_depth = 0;  // re-entrancy guard (HIP calling itself through the PLT)

void logf(int level, const char* fmt, ...) {
  if (g.log < level) return;
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  fprintf(stderr, "[gpushare-hipquota %d] %s\n", (int)getpid(), buf);
}

// ---- real symbol resolution ---------------------------------------------------------------
void* g_hip_handle = nullptr;

int find_hip_cb(struct dl_phdr_info* info, size_t, void* data) {
  if (info->dlpi_name && strstr(info->dlpi_name, "libamdhip64.so")) {
    *static_cast<const char**>(data) = info->dlpi_name;
    return 1;
  }
  return 0;
}

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

#define REAL(ret, name, ...)                                                   \
  using name##_t = ret (*)(__VA_ARGS__);                                       \
  name##_t real_##name() {                                                     \
    static std::atomic<name##_t> fn{nullptr};                                  \
    name##_t f = fn.load(std::memory_order_acquire);                           \
    if (!f) {                                                                  \
      f = reinterpret_cast<name##_t>(resolve(#name));                          \
      fn.store(f, std::memory_order_release);                                  \
    }                                                                          \
    return f;                                                                  \
  }

REAL(hipError_t, hipMalloc, void**, size_t)
REAL(hipError_t, hipExtMallocWithFlags, void**, size_t, unsigned int)
REAL(hipError_t, hipMallocManaged, void**, size_t, unsigned int)
REAL(hipError_t, hipMallocAsync, void**, size_t, hipStream_t)
REAL(hipError_t, hipMallocFromPoolAsync, void**, size_t, hipMemPool_t, hipStream_t)
REAL(hipError_t, hipMallocPitch, void**, size_t*, size_t, size_t)
REAL(hipError_t, hipMalloc3D, hipPitchedPtr*, hipExtent)
REAL(hipError_t, hipFree, void*)
REAL(hipError_t, hipFreeAsync, void*, hipStream_t)
REAL(hipError_t, hipMemCreate, hipMemGenericAllocationHandle_t*, size_t, const hipMemAllocationProp*,
     unsigned long long)
REAL(hipError_t, hipMemRelease, hipMemGenericAllocationHandle_t)
REAL(hipError_t, hipMemGetInfo, size_t*, size_t*)
REAL(hipError_t, hipDeviceTotalMem, size_t*, hipDevice_t)
REAL(hipError_t, hipGetDevicePropertiesR0600, hipDeviceProp_tR0600*, int)
REAL(hipError_t, hipGetDevicePropertiesR0000, hipDeviceProp_tR0000*, int)
REAL(hipError_t, hipGetDeviceProperties, hipDeviceProp_tR0000*, int)

// ---- pointer table (sharded) ---------------------------------------------------------------
struct Shard {
  std::mutex mu;
  std::unordered_map<uintptr_t, uint64_t> m;
};
Shard g_shards[64];

Shard& shard_of(uintptr_t k) { return g_shards[(k >> 21) & 63]; }

void track(uintptr_t k, uint64_t charge) {
  Shard& s = shard_of(k);
  std::lock_guard<std::mutex> lk(s.mu);
  s.m[k] = charge;
}

uint64_t untrack(uintptr_t k) {
  Shard& s = shard_of(k);
  std::lock_guard<std::mutex> lk(s.mu);
  auto it = s.m.find(k);
  if (it == s.m.end()) return 0;
  uint64_t c = it->second;
  s.m.erase(it);
  return c;
}

// ---- ledger --------------------------------------------------------------------------------
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

bool charge(uint64_t bytes) {
  LedgerShm* L = g.ledger;
  bool reclaimed = false;
  uint64_t cur = L->total.load();
  for (;;) {
    if (cur + bytes > g.quota) {
      if (!reclaimed && reclaim_dead(L) > 0) {
        reclaimed = true;
        cur = L->total.load();
        continue;
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
  if (!bytes) return;
  if (g.slot >= 0) g.ledger->slots[g.slot].used.fetch_sub(bytes);
  g.ledger->total.fetch_sub(bytes);
}

uint64_t round_up(uint64_t n, uint64_t g_) { return g_ ? (n + g_ - 1) / g_ * g_ : n; }
uint64_t charge_of(size_t n) { return n == 0 ? 0 : round_up((uint64_t)n, g.granule); }

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  unsigned long long x = strtoull(v, &end, 10);
  return (end && end != v) ? (uint64_t)x : dflt;
}

void release_slot_at_exit() {
  if (!g.enabled || !g.ledger || g.slot < 0) return;
  Slot& s = g.ledger->slots[g.slot];
  uint64_t u = s.used.exchange(0);
  g.ledger->total.fetch_sub(u);
  s.pid.store(0);
  g.slot = -1;
}

void atfork_child() {
  if (g.enabled && g.ledger) g.slot = acquire_slot(g.ledger);  // the child is a new process
}

void init() {
  g.log = (int)env_u64("GPUSHARE_SHIM_LOG", 0);
  const char* dis = getenv("CGPU_DISABLE");
  if (dis && !strcmp(dis, "true")) {
    logf(1, "CGPU_DISABLE=true: quota enforcement off");
    return;
  }
  g.granule = env_u64("GPUSHARE_ALLOC_GRANULE", kDefaultGranule);
  uint64_t q = env_u64("GPUSHARE_QUOTA_BYTES", 0);
  if (!q) {
    uint64_t ctr = env_u64("ALIYUN_COM_GPU_MEM_CONTAINER", 0), dev = env_u64("ALIYUN_COM_GPU_MEM_DEV", 0);
    if (!ctr || !dev) {
      logf(1, "no quota configured: pass-through");
      return;
    }
    size_t fr = 0, tot = 0;
    t_depth++;
    hipError_t e = real_hipMemGetInfo() ? real_hipMemGetInfo()(&fr, &tot) : hipErrorNotInitialized;
    t_depth--;
    if (e != hipSuccess || tot == 0) {
      logf(0, "cannot read device memory (err %d): pass-through", (int)e);
      return;
    }
    q = (uint64_t)((__uint128_t)tot * ctr / dev);
    if (q > tot) q = tot;
  }
  g.quota = q;
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
      void* p = mmap(nullptr, sizeof(LedgerShm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (p != MAP_FAILED) {
        g.ledger = static_cast<LedgerShm*>(p);
        uint64_t zero = 0;  // first process initialises; ftruncate zero-fills
        if (g.ledger->magic.compare_exchange_strong(zero, kMagic)) g.ledger->quota.store(q);
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
  g.quota = g.ledger->quota.load() ? g.ledger->quota.load() : q;
  g.slot = acquire_slot(g.ledger);
  g.enabled = true;
  atexit(release_slot_at_exit);
  pthread_atfork(nullptr, nullptr, atfork_child);
  logf(1, "quota %llu bytes (%.2f GiB), granule %llu, ledger %s slot %d", (unsigned long long)g.quota,
       (double)g.quota / (1ull << 30), (unsigned long long)g.granule, g.ledger_name[0] ? g.ledger_name : "(local)",
       g.slot);
}

inline bool active() {
  std::call_once(g_once, init);
  return g.enabled && t_depth == 0;
}

struct Depth {
  Depth() { ++t_depth; }
  ~Depth() { --t_depth; }
};

hipError_t deny(size_t n) {
  logf(1, "deny %zu bytes: used %llu of %llu", n, (unsigned long long)g.ledger->total.load(),
       (unsigned long long)g.quota);
  return hipErrorOutOfMemory;
}

template <class F>
hipError_t guarded_alloc(void** ptr, size_t size, F&& call) {
  if (!active()) return call();
  uint64_t c = charge_of(size);
  if (c && !charge(c)) {
    if (ptr) *ptr = nullptr;
    return deny(size);
  }
  Depth d;
  hipError_t e = call();
  if (e != hipSuccess || !ptr || !*ptr) {
    uncharge(c);
    return e;
  }
  track((uintptr_t)*ptr, c);
  logf(2, "alloc %zu -> %p (charge %llu, used %llu)", size, *ptr, (unsigned long long)c,
       (unsigned long long)g.ledger->total.load());
  return e;
}

}  // namespace

// ---- interposed API ------------------------------------------------------------------------
GS_EXPORT hipError_t hipMalloc(void** ptr, size_t size) {
  auto f = real_hipMalloc();
  if (!f) return hipErrorNotInitialized;
  return guarded_alloc(ptr, size, [&] { return f(ptr, size); });
}

GS_EXPORT hipError_t hipExtMallocWithFlags(void** ptr, size_t size, unsigned int flags) {
  auto f = real_hipExtMallocWithFlags();
  if (!f) return hipErrorNotInitialized;
  return guarded_alloc(ptr, size, [&] { return f(ptr, size, flags); });
}

GS_EXPORT hipError_t hipMallocManaged(void** ptr, size_t size, unsigned int flags) {
  auto f = real_hipMallocManaged();
  if (!f) return hipErrorNotInitialized;
  return guarded_alloc(ptr, size, [&] { return f(ptr, size, flags); });
}

GS_EXPORT hipError_t hipMallocAsync(void** ptr, size_t size, hipStream_t stream) {
  auto f = real_hipMallocAsync();
  if (!f) return hipErrorNotInitialized;
  return guarded_alloc(ptr, size, [&] { return f(ptr, size, stream); });
}

GS_EXPORT hipError_t hipMallocFromPoolAsync(void** ptr, size_t size, hipMemPool_t pool, hipStream_t stream) {
  auto f = real_hipMallocFromPoolAsync();
  if (!f) return hipErrorNotInitialized;
  return guarded_alloc(ptr, size, [&] { return f(ptr, size, pool, stream); });
}

GS_EXPORT hipError_t hipMallocPitch(void** ptr, size_t* pitch, size_t width, size_t height) {
  auto f = real_hipMallocPitch();
  if (!f) return hipErrorNotInitialized;
  if (!active()) return f(ptr, pitch, width, height);
  hipError_t e;
  {
    Depth d;
    e = f(ptr, pitch, width, height);
  }
  if (e != hipSuccess || !ptr || !*ptr) return e;
  uint64_t c = charge_of(*pitch * height);
  if (!charge(c)) {
    Depth d;
    if (auto fr = real_hipFree()) fr(*ptr);
    *ptr = nullptr;
    return deny(*pitch * height);
  }
  track((uintptr_t)*ptr, c);
  return e;
}

GS_EXPORT hipError_t hipMalloc3D(hipPitchedPtr* pp, hipExtent ext) {
  auto f = real_hipMalloc3D();
  if (!f) return hipErrorNotInitialized;
  if (!active()) return f(pp, ext);
  hipError_t e;
  {
    Depth d;
    e = f(pp, ext);
  }
  if (e != hipSuccess || !pp || !pp->ptr) return e;
  uint64_t c = charge_of(pp->pitch * ext.height * ext.depth);
  if (!charge(c)) {
    Depth d;
    if (auto fr = real_hipFree()) fr(pp->ptr);
    pp->ptr = nullptr;
    return deny(pp->pitch * ext.height * ext.depth);
  }
  track((uintptr_t)pp->ptr, c);
  return e;
}

GS_EXPORT hipError_t hipFree(void* ptr) {
  auto f = real_hipFree();
  if (!f) return hipErrorNotInitialized;
  if (!active() || !ptr) return f(ptr);
  hipError_t e;
  {
    Depth d;
    e = f(ptr);
  }
  if (e == hipSuccess) uncharge(untrack((uintptr_t)ptr));
  return e;
}

GS_EXPORT hipError_t hipFreeAsync(void* ptr, hipStream_t stream) {
  auto f = real_hipFreeAsync();
  if (!f) return hipErrorNotInitialized;
  if (!active() || !ptr) return f(ptr, stream);
  hipError_t e;
  {
    Depth d;
    e = f(ptr, stream);
  }
  if (e == hipSuccess) uncharge(untrack((uintptr_t)ptr));
  return e;
}

GS_EXPORT hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* handle, size_t size,
                                  const hipMemAllocationProp* prop, unsigned long long flags) {
  auto f = real_hipMemCreate();
  if (!f) return hipErrorNotInitialized;
  if (!active()) return f(handle, size, prop, flags);
  uint64_t c = charge_of(size);
  if (c && !charge(c)) return deny(size);
  hipError_t e;
  {
    Depth d;
    e = f(handle, size, prop, flags);
  }
  if (e != hipSuccess || !handle) {
    uncharge(c);
    return e;
  }
  track((uintptr_t)*handle, c);
  return e;
}

GS_EXPORT hipError_t hipMemRelease(hipMemGenericAllocationHandle_t handle) {
  auto f = real_hipMemRelease();
  if (!f) return hipErrorNotInitialized;
  if (!active()) return f(handle);
  hipError_t e;
  {
    Depth d;
    e = f(handle);
  }
  if (e == hipSuccess) uncharge(untrack((uintptr_t)handle));
  return e;
}

GS_EXPORT hipError_t hipMemGetInfo(size_t* free_b, size_t* total_b) {
  auto f = real_hipMemGetInfo();
  if (!f) return hipErrorNotInitialized;
  hipError_t e;
  {
    Depth d;  // init() may call the real hipMemGetInfo itself
    e = f(free_b, total_b);
  }
  if (e != hipSuccess || !active()) return e;
  uint64_t used = g.ledger->total.load();
  uint64_t left = used >= g.quota ? 0 : g.quota - used;
  if (free_b && *free_b > left) *free_b = (size_t)left;
  if (total_b) *total_b = (size_t)g.quota;
  return e;
}

GS_EXPORT hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t dev) {
  auto f = real_hipDeviceTotalMem();
  if (!f) return hipErrorNotInitialized;
  hipError_t e = f(bytes, dev);
  if (e == hipSuccess && active() && bytes && *bytes > g.quota) *bytes = (size_t)g.quota;
  return e;
}

GS_EXPORT hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int dev) {
  auto f = real_hipGetDevicePropertiesR0600();
  if (!f) return hipErrorNotInitialized;
  hipError_t e = f(prop, dev);
  if (e == hipSuccess && active() && prop && prop->totalGlobalMem > g.quota) prop->totalGlobalMem = g.quota;
  return e;
}

GS_EXPORT hipError_t hipGetDevicePropertiesR0000(hipDeviceProp_tR0000* prop, int dev) {
  auto f = real_hipGetDevicePropertiesR0000();
  if (!f) return hipErrorNotInitialized;
  hipError_t e = f(prop, dev);
  if (e == hipSuccess && active() && prop && prop->totalGlobalMem > g.quota) prop->totalGlobalMem = g.quota;
  return e;
}

GS_EXPORT hipError_t hipGetDeviceProperties(hipDeviceProp_tR0000* prop, int dev) {
  auto f = real_hipGetDeviceProperties();
  if (!f) return hipErrorNotInitialized;
  hipError_t e = f(prop, dev);
  if (e == hipSuccess && active() && prop && prop->totalGlobalMem > g.quota) prop->totalGlobalMem = g.quota;
  return e;
}

// ---- introspection (tests, metrics) --------------------------------------------------------
GS_EXPORT int gpushare_shim_stats(uint64_t* used, uint64_t* quota, uint64_t* denied, uint64_t* peak) {
  std::call_once(g_once, init);
  if (!g.enabled) return 0;
  if (used) *used = g.ledger->total.load();
  if (quota) *quota = g.quota;
  if (denied) *denied = g.ledger->denied.load();
  if (peak) *peak = g.ledger->peak.load();
  return 1;
}

GS_EXPORT uint64_t gpushare_shim_granule() { return g.granule; }
