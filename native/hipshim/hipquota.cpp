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
// Enforcement point (default, GPUSHARE_SHIM_MODE=kfd): the KFD boundary. Every byte of HBM a
// process owns is created by one ioctl on /dev/kfd — AMDKFD_IOC_ALLOC_MEMORY_OF_GPU with the
// VRAM flag — issued by ROCr (libhsa-runtime64 imports ioctl from libc through its PLT, so a
// preloaded ioctl sees it) and released by AMDKFD_IOC_FREE_MEMORY_OF_GPU. Charging there
// covers what the HIP entry points cannot see: hipMallocAsync pools that keep memory after
// hipFreeAsync (charged until the pool trims), hipMallocArray / 3D arrays, scratch (private
// segment) buffers, code objects, queue and staging buffers allocated inside the runtime, and
// programs that call HSA directly. The charge is the physical allocation KFD hands out (ROCr
// grabs 2 MiB fragments and sub-allocates), so no rounding model is needed. Over quota the
// ioctl fails with ENOMEM, exactly as when HBM runs out: ROCr trims its caches and retries,
// then reports HSA_STATUS_ERROR_OUT_OF_RESOURCES / hipErrorOutOfMemory.
//
// hipMemGetInfo / hipDeviceTotalMem / hipGetDeviceProperties are also interposed so frameworks
// see the quota as the device total and the quota's remainder as free memory.
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
// The render node is the second way to HBM: a container is handed /dev/dri/renderD<n> (for
// libdrm / Mesa / video) and DRM_IOCTL_AMDGPU_GEM_CREATE with the VRAM domain allocates HBM
// there, outside KFD. In kfd mode those buffer objects are charged too. GEM handles belong to
// the DRM *file* (one open file description, shared by dup'ed and inherited fds), not to an
// fd number, so charges are keyed by the file's DRM client id (amdgpu fdinfo
// "drm-client-id") and a handle: DRM_IOCTL_GEM_CLOSE on any fd of that file releases one;
// closing an fd releases the file's charges only when no fd of any process this shim can see
// (/proc: the container's processes) still refers to that client — otherwise the client
// lingers and is re-checked when another fd of it closes and before any denial. A charged
// VRAM handle cannot be exported as a dma-buf (DRM_IOCTL_PRIME_HANDLE_TO_FD fails with EACCES),
// because the dma-buf would keep the HBM alive after GEM_CLOSE; GPUSHARE_SHIM_PRIME=keep
// allows the export and keeps the handle charged until its DRM file is gone.
//
// Limits (documented, by construction): enforcement is cooperative — a process that drops
// LD_PRELOAD or issues the ioctl through a raw syscall is not charged. Memory imported from
// another process (dma-buf / IPC) is charged to its exporter only. KFD allocations issued
// while the shim itself is initialising (the runtime's own start-up, reached from init) pass
// uncharged. A GEM buffer still CPU-mapped after its GEM_CLOSE (the mapping holds it), and a
// DRM file held only by a process the shim cannot read in /proc, are not followed; the node's
// quota watchdog (amdgpu fdinfo / VRAM usage, quota/watchdog.py) is the backstop there.
//
// The library does not link libamdhip64 or libhsa-runtime64: the real entry points are
// resolved at run time from whichever runtime the process loaded (PyTorch ships its own copy).
// It is linked with -static-libstdc++ -static-libgcc so it loads into any tenant image.

#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <hip/hip_deprecated.h>

#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <link.h>
#include <poll.h>
#include <pthread.h>
#include <signal.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/sysmacros.h>
#include <unistd.h>

#include <atomic>
#include <new>

// Symbol versions pinned to the x86-64 glibc baseline (2.2.5) so the shim loads into tenant
// images with an old glibc (it is linked against this image's 2.35, where these moved into
// libc proper under GLIBC_2.34); libdl/librt/libpthread stay NEEDED for those images.
__asm__(".symver dlsym,dlsym@GLIBC_2.2.5");
__asm__(".symver dlopen,dlopen@GLIBC_2.2.5");
__asm__(".symver shm_open,shm_open@GLIBC_2.2.5");
__asm__(".symver pthread_once,pthread_once@GLIBC_2.2.5");
__asm__(".symver memcpy,memcpy@GLIBC_2.2.5");

#undef hipGetDeviceProperties

#define GS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

constexpr uint64_t kMagic = 0x67707573686172ULL;  // "gpushar"
constexpr int kSlots = 256;
constexpr uint64_t kDefaultGranule = 2ull << 20;

// ---- KFD uapi (linux/kfd_ioctl.h, stable since KFD 1.0; mirrored so the shim builds without
// kernel headers and matches any ROCr) ----------------------------------------------------------
struct KfdAllocArgs {   // struct kfd_ioctl_alloc_memory_of_gpu_args
  uint64_t va_addr;
  uint64_t size;
  uint64_t handle;
  uint64_t mmap_offset;
  uint32_t gpu_id;
  uint32_t flags;
};
struct KfdFreeArgs {    // struct kfd_ioctl_free_memory_of_gpu_args
  uint64_t handle;
};
constexpr uint32_t kKfdVram = 1u << 0;  // KFD_IOC_ALLOC_MEM_FLAGS_VRAM
// _IOC(dir, 'K', nr, size): dir bits 30-31 (1 write, 2 read), size bits 16-29, type 8-15, nr 0-7
constexpr unsigned long kfd_ioc(unsigned dir, unsigned nr, unsigned size) {
  return ((unsigned long)dir << 30) | ((unsigned long)size << 16) | ((unsigned long)'K' << 8) | nr;
}
constexpr unsigned long kIocAlloc = kfd_ioc(3, 0x16, sizeof(KfdAllocArgs));  // AMDKFD_IOWR(0x16)
constexpr unsigned long kIocFree = kfd_ioc(1, 0x17, sizeof(KfdFreeArgs));    // AMDKFD_IOW(0x17)
static_assert(sizeof(KfdAllocArgs) == 40 && sizeof(KfdFreeArgs) == 8, "KFD uapi layout");
struct KfdUnmapArgs {   // struct kfd_ioctl_unmap_memory_from_gpu_args
  uint64_t handle;
  uint64_t device_ids_array_ptr;
  uint32_t n_devices;
  uint32_t n_success;
};
struct KfdImportArgs {  // struct kfd_ioctl_import_dmabuf_args
  uint64_t va_addr;
  uint64_t handle;
  uint32_t gpu_id;
  uint32_t dmabuf_fd;
};
constexpr unsigned long kIocUnmap = kfd_ioc(3, 0x19, sizeof(KfdUnmapArgs));    // AMDKFD_IOWR(0x19)
constexpr unsigned long kIocImport = kfd_ioc(3, 0x1D, sizeof(KfdImportArgs));  // AMDKFD_IOWR(0x1D)
static_assert(sizeof(KfdUnmapArgs) == 24 && sizeof(KfdImportArgs) == 24, "KFD uapi layout");

// ---- amdgpu DRM uapi (drm/amdgpu_drm.h, drm/drm.h) -----------------------------------------
struct DrmGemCreateIn {   // union drm_amdgpu_gem_create: in {bo_size, alignment, domains, domain_flags}
  uint64_t bo_size;       //                              out {u32 handle, u32 _pad} (overlays bo_size)
  uint64_t alignment;
  uint64_t domains;
  uint64_t domain_flags;
};
struct DrmGemClose {      // struct drm_gem_close
  uint32_t handle;
  uint32_t pad;
};
constexpr unsigned long drm_ioc(unsigned dir, unsigned nr, unsigned size) {
  return ((unsigned long)dir << 30) | ((unsigned long)size << 16) | ((unsigned long)'d' << 8) | nr;
}
constexpr unsigned long kDrmGemCreate = drm_ioc(3, 0x40 + 0x00, sizeof(DrmGemCreateIn));  // DRM_IOCTL_AMDGPU_GEM_CREATE
constexpr unsigned long kDrmGemClose = drm_ioc(1, 0x09, sizeof(DrmGemClose));              // DRM_IOCTL_GEM_CLOSE
constexpr uint64_t kAmdgpuDomainVram = 0x4;                                               // AMDGPU_GEM_DOMAIN_VRAM
static_assert(sizeof(DrmGemCreateIn) == 32 && sizeof(DrmGemClose) == 8, "DRM uapi layout");
struct DrmPrimeHandle {    // struct drm_prime_handle
  uint32_t handle, flags;
  int32_t fd;
};
constexpr unsigned long kDrmPrimeHandleToFd = drm_ioc(3, 0x2d, sizeof(DrmPrimeHandle));  // DRM_IOCTL_PRIME_HANDLE_TO_FD
static_assert(sizeof(DrmPrimeHandle) == 12, "DRM uapi layout");
constexpr int kMaxDrmFd = 4096;
// Table key of a GEM handle: bit 63 set (KFD handles are gpu_id << 32 | idr, bit 63 clear),
// bit 62 = kept after a dma-buf export (GEM_CLOSE does not release it), bits 32-61 = the DRM
// client key (client id, or kFdClient | fd when the kernel reports none), bits 0-31 = handle.
constexpr uint64_t kGemBit = 1ull << 63, kStickyBit = 1ull << 62;
constexpr uint64_t kClientMask = (1ull << 30) - 1, kFdClient = 1ull << 29;
inline uint64_t gem_key(uint64_t client, uint32_t h) { return kGemBit | (client & kClientMask) << 32 | h; }
inline uint64_t client_of_key(uint64_t k) { return k >> 32 & kClientMask; }

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

enum Mode { kModeKfd = 0, kModeHip = 1 };

struct State {
  bool enabled = false;
  int mode = kModeKfd;
  int log = 0;
  int diag = 0;
  std::atomic<uint64_t> quota{0};   // 0 in kfd mode until the first VRAM allocation names its GPU
  uint64_t ctr = 0, dev = 0;        // container / device units when the quota is derived
  uint64_t granule = kDefaultGranule;
  LedgerShm* ledger = nullptr;
  LedgerShm local{};  // used when no shared ledger is configured
  int slot = -1;
  char ledger_name[128] = {0};
};

State g;
pthread_once_t g_once = PTHREAD_ONCE_INIT;
// init() in progress (any thread): an ioctl reached from it (the runtime starting up under a
// HIP call the shim makes) must not wait on the once-control held by that same init
std::atomic<bool> g_initializing{false};
std::atomic<int> g_env_mode{-1};          // GPUSHARE_SHIM_MODE read without initialising
std::atomic<uint64_t> g_drm_client[kMaxDrmFd];  // fd -> its DRM client key + 1 (0: no charged GEM handles)
std::atomic<int> g_gem_live{0};                  // charged GEM handles in this process (fast path skip)
struct Lingering {                               // clients whose charged fd closed while still referred to
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  uint64_t client[64];
  int n = 0;
};
Lingering g_linger;
std::atomic<bool> g_released{false};  // set by the atexit handler (see release_slot_at_exit)
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

using ioctl_t = int (*)(int, unsigned long, ...);
std::atomic<ioctl_t> g_real_ioctl{nullptr};

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
struct Shard {
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  uint64_t* keys = nullptr;
  uint64_t* vals = nullptr;
  size_t cap = 0, used = 0;  // used counts live + deleted slots
};
Shard g_shards[64];
constexpr uint64_t kEmpty = 0, kDeleted = ~0ull;

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

int linger_gc();

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

uint64_t round_up(uint64_t n, uint64_t g_) { return g_ ? (n + g_ - 1) / g_ * g_ : n; }
uint64_t charge_of(size_t n) { return n == 0 ? 0 : round_up((uint64_t)n, g.granule); }

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  unsigned long long x = strtoull(v, &end, 10);
  return (end && end != v) ? (uint64_t)x : dflt;
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
  for (auto& fl : g_drm_client) fl.store(0, std::memory_order_relaxed);   // the parent's GEM handles are the parent's
  g_gem_live.store(0);
  pthread_mutex_init(&g_linger.mu, nullptr);
  g_linger.n = 0;
  g.slot = acquire_slot(g.ledger);
}

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

void init_body();

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

void init() {
  g_initializing.store(true);
  init_body();
  g_initializing.store(false);
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

inline bool enabled() {
  pthread_once(&g_once, init);
  return g.enabled;
}

// HIP-API accounting applies in hip mode only (kfd mode charges below, at the ioctl).
inline bool hip_active() { return enabled() && g.mode == kModeHip && t_depth == 0; }

struct Depth {
  Depth() { ++t_depth; }
  ~Depth() { --t_depth; }
};

hipError_t deny(size_t n) {
  logf(1, "deny %zu bytes: used %llu of %llu", n, (unsigned long long)g.ledger->total.load(),
       (unsigned long long)g.quota.load());
  return hipErrorOutOfMemory;
}

template <class F>
hipError_t guarded_alloc(void** ptr, size_t size, F&& call) {
  if (!hip_active()) return call();
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
  track((uint64_t)(uintptr_t)*ptr, c);
  logf(2, "alloc %zu -> %p (charge %llu, used %llu)", size, *ptr, (unsigned long long)c,
       (unsigned long long)g.ledger->total.load());
  return e;
}

// ---- KFD boundary --------------------------------------------------------------------------
int kfd_alloc(ioctl_t f, int fd, unsigned long req, KfdAllocArgs* a) {
  if (!g.quota.load(std::memory_order_relaxed)) set_quota_from_device_bytes(kfd_vram_bytes(a->gpu_id));
  uint64_t c = a->size;
  if (!charge(c)) {
    logf(1, "deny VRAM %llu bytes on gpu_id %u: used %llu of %llu", (unsigned long long)c, a->gpu_id,
         (unsigned long long)g.ledger->total.load(), (unsigned long long)g.quota.load());
    errno = ENOMEM;
    return -1;
  }
  int r = f(fd, req, a);
  if (r != 0) {
    int err = errno;
    uncharge(c);
    errno = err;
    return r;
  }
  track(a->handle, c);
  logf(2, "kfd alloc %llu bytes (flags 0x%x) -> handle 0x%llx, used %llu", (unsigned long long)c, a->flags,
       (unsigned long long)a->handle, (unsigned long long)g.ledger->total.load());
  return r;
}

// ---- render node (amdgpu GEM) ---------------------------------------------------------------
// /proc, or GPUSHARE_SHIM_PROC_ROOT (tests: a synthetic tree of <pid>/fd and <pid>/fdinfo)
const char* proc_root() {
  static const char* r = nullptr;
  if (!r) {
    const char* v = getenv("GPUSHARE_SHIM_PROC_ROOT");
    r = (v && *v) ? v : "/proc";
  }
  return r;
}

// "drm-client-id" of <root>/<pid>/fdinfo/<fd> (0 = none: not a DRM file, or an old kernel).
uint64_t read_client_id(const char* path) {
  int f = open(path, O_RDONLY | O_CLOEXEC);
  if (f < 0) return 0;
  char buf[2048];
  ssize_t n = read(f, buf, sizeof buf - 1);
  syscall(SYS_close, f);  // not through the interposed close (it may call back in here)
  if (n <= 0) return 0;
  buf[n] = 0;
  const char* p = strstr(buf, "drm-client-id:");
  return p ? strtoull(p + 14, nullptr, 10) : 0;
}

// The DRM client key of this process's fd: the kernel's client id (shared by every fd of one
// open file description), or kFdClient | fd when the kernel does not report one.
uint64_t client_key_of(int fd) {
  char path[96];
  snprintf(path, sizeof path, "%s/%d/fdinfo/%d", proc_root(), (int)getpid(), fd);
  uint64_t id = read_client_id(path);
  return id ? (id & kClientMask & ~kFdClient) : (kFdClient | (uint64_t)fd);
}

// Does any fd of any process visible in /proc still refer to DRM client `key`?
bool client_alive(uint64_t key) {
  if (key & kFdClient) return false;  // no client ids on this kernel: the fd was the file
  DIR* d = opendir(proc_root());
  if (!d) return true;  // cannot tell: keep the charge
  bool alive = false;
  char path[160], link[64];
  while (!alive) {
    struct dirent* e = readdir(d);
    if (!e) break;
    if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
    snprintf(path, sizeof path, "%s/%s/fd", proc_root(), e->d_name);
    DIR* fds = opendir(path);
    if (!fds) continue;  // exited, or not ours to read
    while (!alive) {
      struct dirent* f = readdir(fds);
      if (!f) break;
      if (f->d_name[0] < '0' || f->d_name[0] > '9') continue;
      snprintf(path, sizeof path, "%s/%s/fd/%s", proc_root(), e->d_name, f->d_name);
      ssize_t n = readlink(path, link, sizeof link - 1);
      if (n <= 0) continue;
      link[n] = 0;
      if (strncmp(link, "/dev/dri/", 9) != 0) continue;
      snprintf(path, sizeof path, "%s/%s/fdinfo/%s", proc_root(), e->d_name, f->d_name);
      uint64_t id = read_client_id(path);
      alive = id && (id & kClientMask & ~kFdClient) == key;
    }
    closedir(fds);
  }
  closedir(d);
  return alive;
}

// Release every charged GEM handle (sticky ones included) of DRM client `key`.
uint64_t release_client(uint64_t key) {
  uint64_t freed = 0;
  int handles = 0;
  for (auto& s : g_shards) {
    pthread_mutex_lock(&s.mu);
    for (size_t i = 0; i < s.cap; ++i) {
      uint64_t k = s.keys[i];
      if (k != kEmpty && k != kDeleted && (k & kGemBit) && client_of_key(k) == key) {
        freed += s.vals[i];
        s.keys[i] = kDeleted;
        ++handles;
      }
    }
    pthread_mutex_unlock(&s.mu);
  }
  g_gem_live.fetch_sub(handles);
  uncharge(freed);
  logf(2, "DRM client %llu gone: %llu GEM bytes released", (unsigned long long)key, (unsigned long long)freed);
  return freed;
}

void linger_add(uint64_t key) {
  pthread_mutex_lock(&g_linger.mu);
  bool have = false;
  for (int i = 0; i < g_linger.n; ++i) have |= g_linger.client[i] == key;
  if (!have && g_linger.n < 64) g_linger.client[g_linger.n++] = key;
  pthread_mutex_unlock(&g_linger.mu);
  if (!have) logf(1, "DRM client %llu still referred to after its fd closed: GEM charges kept", (unsigned long long)key);
}

// Re-check lingering clients; returns how many were released.
bool linger_has(uint64_t key) {
  pthread_mutex_lock(&g_linger.mu);
  bool have = false;
  for (int i = 0; i < g_linger.n; ++i) have |= g_linger.client[i] == key;
  pthread_mutex_unlock(&g_linger.mu);
  return have;
}

int linger_gc() {
  pthread_mutex_lock(&g_linger.mu);
  int n = g_linger.n, released = 0;
  uint64_t keys[64];
  memcpy(keys, g_linger.client, sizeof(uint64_t) * (size_t)n);
  pthread_mutex_unlock(&g_linger.mu);
  if (!n) return 0;
  for (int i = 0; i < n; ++i) {
    if (client_alive(keys[i])) continue;
    release_client(keys[i]);
    ++released;
    pthread_mutex_lock(&g_linger.mu);
    for (int j = 0; j < g_linger.n; ++j)
      if (g_linger.client[j] == keys[i]) {
        g_linger.client[j] = g_linger.client[--g_linger.n];
        break;
      }
    pthread_mutex_unlock(&g_linger.mu);
  }
  return released;
}

int gem_create(ioctl_t f, int fd, unsigned long req, DrmGemCreateIn* a) {
  if (!(a->domains & kAmdgpuDomainVram) || fd < 0 || fd >= kMaxDrmFd) return f(fd, req, a);
  uint64_t c = round_up(a->bo_size, 4096);
  if (!g.quota.load(std::memory_order_relaxed)) set_quota_from_device_bytes(render_vram_bytes(fd));
  if (!g.quota.load(std::memory_order_relaxed)) {
    logf(1, "GEM VRAM %llu bytes before the quota is known: not charged", (unsigned long long)c);
    return f(fd, req, a);
  }
  if (!charge(c)) {
    logf(1, "deny GEM VRAM %llu bytes on fd %d: used %llu of %llu", (unsigned long long)c, fd,
         (unsigned long long)g.ledger->total.load(), (unsigned long long)g.quota.load());
    errno = ENOMEM;
    return -1;
  }
  int r = f(fd, req, a);
  if (r != 0) {
    int err = errno;
    uncharge(c);
    errno = err;
    return r;
  }
  uint32_t h = reinterpret_cast<DrmGemClose*>(a)->handle;   // out.handle overlays bo_size
  uint64_t key = client_key_of(fd);                          // read each time: fd numbers are reused
  g_drm_client[fd].store(key + 1, std::memory_order_relaxed);
  g_gem_live.fetch_add(1);
  track(gem_key(key, h), c);
  logf(2, "gem create %llu bytes VRAM on fd %d (client %llu) -> handle %u, used %llu", (unsigned long long)c, fd,
       (unsigned long long)key, h, (unsigned long long)g.ledger->total.load());
  return r;
}

// The DRM client key of a render fd a GEM ioctl names (recorded at create, else read).
uint64_t gem_client(int fd) {
  uint64_t k = fd >= 0 && fd < kMaxDrmFd ? g_drm_client[fd].load(std::memory_order_relaxed) : 0;
  return k ? k - 1 : client_key_of(fd);
}

int gem_close(ioctl_t f, int fd, unsigned long req, DrmGemClose* a) {
  uint32_t gh = a->handle;
  int r = f(fd, req, a);
  if (r == 0 && g_gem_live.load(std::memory_order_relaxed) > 0) {
    uint64_t c = untrack(gem_key(gem_client(fd), gh));
    if (c) {
      g_gem_live.fetch_sub(1);
      uncharge(c);
      logf(2, "gem close fd %d handle %u -> %llu bytes", fd, gh, (unsigned long long)c);
    }
  }
  return r;
}

// Exporting a charged VRAM handle as a dma-buf would let the HBM outlive GEM_CLOSE uncharged:
// refused (EACCES), or with GPUSHARE_SHIM_PRIME=keep exported and kept charged until the DRM
// file is gone.
int prime_export(ioctl_t f, int fd, unsigned long req, DrmPrimeHandle* a) {
  if (g_gem_live.load(std::memory_order_relaxed) <= 0) return f(fd, req, a);
  uint64_t k = gem_key(gem_client(fd), a->handle);
  uint64_t c = untrack(k);
  if (!c) return f(fd, req, a);
  const char* mode = getenv("GPUSHARE_SHIM_PRIME");
  if (!(mode && !strcmp(mode, "keep"))) {
    track(k, c);
    logf(1, "refused dma-buf export of charged VRAM handle %u on fd %d (GPUSHARE_SHIM_PRIME=keep allows it)",
         a->handle, fd);
    errno = EACCES;
    return -1;
  }
  int r = f(fd, req, a);
  track(r == 0 ? (k | kStickyBit) : k, c);
  if (r == 0) logf(2, "dma-buf export of handle %u: charge kept until its DRM file is gone", a->handle);
  return r;
}

// A closed render fd: the DRM file's GEM handles die with the file, which may still be open
// through a dup'ed or inherited fd — released now if not, else once it is (linger_gc).
void gem_fd_closed(int fd, uint64_t key) {
  for (int i = 0; i < kMaxDrmFd; ++i)
    if (i != fd && g_drm_client[i].load(std::memory_order_relaxed) == key + 1) {
      logf(2, "render fd %d closed: DRM client %llu still open as fd %d", fd, (unsigned long long)key, i);
      return;
    }
  if (client_alive(key)) {
    linger_add(key);
    return;
  }
  release_client(key);
}

// ---- the runtime's KFD imports of broker granules ----
// HIP 7.0 (the runtime PyTorch bundles) never frees the KFD object it creates when it imports a
// dma-buf: after hipMemRelease the granule stays referenced until the process is torn down, and
// the broker cannot lend it to the next pod before that (tools/diag/dmabuf_ref_probe.cpp,
// profiles/r5/dmabuf_refs/). HIP 7.2 frees it at hipMemRelease. So the shim notes the imports the
// runtime makes while the arena imports its granules, and at gpushare_shim_arena_release() frees
// the ones a runtime older than 7.1 left behind.
struct KfdImport {
  uint64_t handle;
  int kfd;
  uint32_t gpu_id;
  bool live;
};
constexpr int kMaxImports = 2048;
KfdImport g_imports[kMaxImports];
int g_nimports = 0;
std::atomic<int> g_imports_live{0};
pthread_mutex_t g_imp_mu = PTHREAD_MUTEX_INITIALIZER;
thread_local bool t_importing = false;  // inside the arena's own import of a granule

void import_note(int kfd, const KfdImportArgs* a) {
  pthread_mutex_lock(&g_imp_mu);
  if (g_nimports < kMaxImports) {
    g_imports[g_nimports++] = {a->handle, kfd, a->gpu_id, true};
    g_imports_live.fetch_add(1, std::memory_order_relaxed);
  }
  pthread_mutex_unlock(&g_imp_mu);
}

void import_forget(uint64_t handle) {
  pthread_mutex_lock(&g_imp_mu);
  for (int i = 0; i < g_nimports; ++i)
    if (g_imports[i].live && g_imports[i].handle == handle) {
      g_imports[i].live = false;
      g_imports_live.fetch_sub(1, std::memory_order_relaxed);
    }
  pthread_mutex_unlock(&g_imp_mu);
}

// free the imports the runtime kept (after it released every arena handle); returns how many
int imports_free_kept(ioctl_t f) {
  int n = 0;
  pthread_mutex_lock(&g_imp_mu);
  for (int i = 0; i < g_nimports; ++i) {
    KfdImport& m = g_imports[i];
    if (!m.live) continue;
    uint32_t dev = m.gpu_id;
    KfdUnmapArgs u{m.handle, reinterpret_cast<uint64_t>(&dev), 1, 0};
    (void)f(m.kfd, kIocUnmap, &u);  // mapped through VMM, not KFD: normally refused, harmless
    KfdFreeArgs fr{m.handle};
    if (f(m.kfd, kIocFree, &fr) == 0) ++n;
    m.live = false;
  }
  g_nimports = 0;
  g_imports_live.store(0, std::memory_order_relaxed);
  pthread_mutex_unlock(&g_imp_mu);
  return n;
}

int ioctl_body(ioctl_t f, int fd, unsigned long req, void* arg);
}  // namespace

// ---- interposed libc ioctl (kfd mode) ------------------------------------------------------
GS_EXPORT int ioctl(int fd, unsigned long req, ...) {
  va_list ap;
  va_start(ap, req);
  void* arg = va_arg(ap, void*);
  va_end(ap);
  ioctl_t f = real_ioctl();
  if (!f) {
    errno = ENOSYS;
    return -1;
  }
  if (req == kIocImport && arg && t_importing) {
    int r = f(fd, req, arg);
    if (r == 0) import_note(fd, static_cast<KfdImportArgs*>(arg));
    return r;
  }
  if (req == kIocFree && arg && g_imports_live.load(std::memory_order_relaxed) > 0) {
    uint64_t h = static_cast<KfdFreeArgs*>(arg)->handle;
    int r = ioctl_body(f, fd, req, arg);
    if (r == 0) import_forget(h);
    return r;
  }
  return ioctl_body(f, fd, req, arg);
}

namespace {
int ioctl_body(ioctl_t f, int fd, unsigned long req, void* arg) {
  // Cheap filters first, and never the once-control while init() runs (the runtime may start
  // up underneath it and allocate through here: waiting on that init would deadlock).
  if ((req != kIocAlloc && req != kIocFree && req != kDrmGemCreate && req != kDrmGemClose &&
       req != kDrmPrimeHandleToFd) || !arg || env_mode() != kModeKfd || g_initializing.load(std::memory_order_acquire))
    return f(fd, req, arg);
  if (req == kIocAlloc && !(static_cast<KfdAllocArgs*>(arg)->flags & kKfdVram)) return f(fd, req, arg);
  if ((req == kDrmGemClose || req == kDrmPrimeHandleToFd) && g_gem_live.load(std::memory_order_relaxed) <= 0)
    return f(fd, req, arg);
  if (!enabled()) return f(fd, req, arg);
  if (req == kDrmGemCreate) return gem_create(f, fd, req, static_cast<DrmGemCreateIn*>(arg));
  if (req == kDrmGemClose) return gem_close(f, fd, req, static_cast<DrmGemClose*>(arg));
  if (req == kDrmPrimeHandleToFd) return prime_export(f, fd, req, static_cast<DrmPrimeHandle*>(arg));
  if (req == kIocAlloc) return kfd_alloc(f, fd, req, static_cast<KfdAllocArgs*>(arg));
  uint64_t h = static_cast<KfdFreeArgs*>(arg)->handle;
  int r = f(fd, req, arg);
  if (r == 0) {
    uint64_t c = untrack(h);
    uncharge(c);
    logf(2, "kfd free handle 0x%llx -> %llu bytes, used %llu", (unsigned long long)h, (unsigned long long)c,
         (unsigned long long)g.ledger->total.load());
  }
  return r;
}
}  // namespace

// ---- interposed libc close (render-node fds with charged GEM handles) ----------------------
using close_t = int (*)(int);

GS_EXPORT int close(int fd) {
  static std::atomic<close_t> real{nullptr};
  close_t f = real.load(std::memory_order_acquire);
  if (!f) {
    f = reinterpret_cast<close_t>(dlsym(RTLD_NEXT, "close"));
    real.store(f, std::memory_order_release);
  }
  if (fd >= 0 && fd < kMaxDrmFd && g_drm_client[fd].load(std::memory_order_relaxed)) {
    // forget the fd before the real close: once closed, another thread may get the same number
    // for a new render fd and charge handles under it
    uint64_t ck = g_drm_client[fd].exchange(0, std::memory_order_acq_rel);
    int r = f(fd);
    if (r != 0 && errno == EBADF) {
      g_drm_client[fd].store(ck, std::memory_order_relaxed);
      return r;
    }
    if (ck) {
      int err = errno;
      gem_fd_closed(fd, ck - 1);
      errno = err;
    }
    return r;
  }
  if (f && fd >= 0 && __atomic_load_n(&g_linger.n, __ATOMIC_RELAXED) > 0) {
    // the last fd of a lingering DRM file (a dup the shim never saw used) may be this one
    uint64_t k = client_key_of(fd);
    int r = f(fd);
    if (r == 0 && !(k & kFdClient) && linger_has(k)) {
      int err = errno;
      linger_gc();
      errno = err;
    }
    return r;
  }
  return f ? f(fd) : (errno = ENOSYS, -1);
}

// ---- HBM broker arena ------------------------------------------------------------------------
// GPUSHARE_HBM_BROKER=<socket> + GPUSHARE_HBM_TOKEN=<token>: the pod's HBM comes from the node's
// HBM broker (native/hbmbroker) instead of fresh driver allocations, so it never waits for
// amdgpu's wipe of a retired pod's memory. At the first hipMalloc the shim takes its grant (the
// fds of its granules, and only those), imports and maps them contiguously, and serves
// hipMalloc/hipFree from that range. The broker connection stays open for the process lifetime:
// its end returns the granules (scrubbed) to the broker. gpushare_shim_arena_release() hands them
// back early, once nothing in the arena is live.
namespace {
REAL(hipError_t, hipMemImportFromShareableHandle, hipMemGenericAllocationHandle_t*, void*,
     hipMemAllocationHandleType)
REAL(hipError_t, hipMemAddressReserve, void**, size_t, size_t, void*, unsigned long long)
REAL(hipError_t, hipMemAddressFree, void*, size_t)
REAL(hipError_t, hipMemMap, void*, size_t, size_t, hipMemGenericAllocationHandle_t, unsigned long long)
REAL(hipError_t, hipMemUnmap, void*, size_t)
REAL(hipError_t, hipMemSetAccess, void*, size_t, const hipMemAccessDesc*, size_t)
REAL(hipError_t, hipGetDevice, int*)
REAL(hipError_t, hipDeviceSynchronize)
REAL(hipError_t, hipRuntimeGetVersion, int*)
REAL(hipError_t, hipGetLastError)
REAL(hipError_t, hipEventCreateWithFlags, hipEvent_t*, unsigned)
REAL(hipError_t, hipEventRecord, hipEvent_t, hipStream_t)
REAL(hipError_t, hipEventQuery, hipEvent_t)
REAL(hipError_t, hipEventSynchronize, hipEvent_t)
REAL(hipError_t, hipEventDestroy, hipEvent_t)
REAL(hipError_t, hipStreamIsCapturing, hipStream_t, hipStreamCaptureStatus*)
REAL(hipError_t, hipDeviceGetDefaultMemPool, hipMemPool_t*, int)
REAL(hipError_t, hipMemGetAllocationPropertiesFromHandle, hipMemAllocationProp*, hipMemGenericAllocationHandle_t)
REAL(hipError_t, hipMemExportToShareableHandle, void*, hipMemGenericAllocationHandle_t, hipMemAllocationHandleType,
     unsigned long long)

constexpr int kArenaMaxGranules = 1024;
constexpr int kArenaMaxExt = 1 << 16;     // free extents
constexpr int kArenaLiveCap = 1 << 17;    // live allocations (open addressing, power of two)

struct Ext {
  uint64_t off, len;
};
struct Live {
  uint64_t off1;  // offset + 1 (0 = empty slot)
  uint64_t len;
  bool tomb;
};

struct Arena {
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  std::atomic<int> state{0};  // 0 untried, 1 active, -1 off (no broker configured, failed or released)
  int sock = -1;
  char* base = nullptr;
  // size: the pod's grant (total granules; charged, and what hipMemGetInfo promises); vsize: the
  // address range reserved for it. A streaming TAKE maps granules [0, n) and is owed [n, total)
  uint64_t size = 0, vsize = 0, gran = 0, used = 0;
  int n = 0, total = 0;
  bool by_address = false;  // how this runtime imports a POSIX fd (see arena_take)
  int rt_version = 0;       // hipRuntimeGetVersion
  hipMemGenericAllocationHandle_t h[kArenaMaxGranules];
  Ext* ext = nullptr;
  int next = 0;
  Live* live = nullptr;
  uint64_t nlive = 0;
  bool charged = false;  // the arena's size is on the pod's ledger
};
Arena g_arena;
int g_dev = 0;  // the arena's device (HIP ordinal in this process)
// where a TAKE's time went (ns): connecting to the broker, waiting for its answer, importing and
// mapping the granules (gpushare_shim_arena_timing); then, for a streaming TAKE, allocations that
// waited for owed granules, importing and mapping those, and MORE messages received
uint64_t g_take_connect_ns = 0, g_take_wait_ns = 0, g_take_map_ns = 0;
uint64_t g_more_wait_ns = 0, g_more_map_ns = 0, g_more_msgs = 0, g_more_waits = 0;
uint64_t g_take_first = 0, g_take_reserve_ns = 0, g_take_access_ns = 0;  // the TAKE's first batch
uint64_t g_first_import_ns = 0, g_first_map_ns = 0;  // the process's first granule
uint64_t g_take_header_ns = 0;                       // TAKE sent -> the broker's answer line

uint64_t mono_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return uint64_t(t.tv_sec) * 1000000000ull + uint64_t(t.tv_nsec);
}

bool arena_configured() {
  static std::atomic<int> c{-1};
  int v = c.load(std::memory_order_relaxed);
  if (v < 0) {
    v = getenv("GPUSHARE_HBM_BROKER") && getenv("GPUSHARE_HBM_TOKEN") ? 1 : 0;
    c.store(v, std::memory_order_relaxed);
  }
  return v == 1;
}

bool recv_line(int s, char* buf, size_t cap) {
  size_t i = 0;
  while (i + 1 < cap) {
    char ch;
    ssize_t r = recv(s, &ch, 1, 0);
    if (r <= 0) return false;
    if (ch == '\n') break;
    buf[i++] = ch;
  }
  buf[i] = 0;
  return true;
}

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
  for (int i = 0; i < k; ++i) {
    uint64_t t0 = mono_ns();
    t_importing = true;
    hipError_t e = by_address ? import_f(&h[i], &fds[i], hipMemHandleTypePosixFileDescriptor)
                              : import_f(&h[i], reinterpret_cast<void*>(static_cast<intptr_t>(fds[i])),
                                         hipMemHandleTypePosixFileDescriptor);
    t_importing = false;
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
  return f && f(va, len, &acc, 1) == hipSuccess;
}

// where the last arena release spent its time (ns): device sync, unmaps, address free, handle
// releases, the KFD frees of kept imports (gpushare_shim_arena_release_timing)
uint64_t g_rel_ns[5];

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
  uint64_t t4 = mono_ns();
  g_rel_ns[0] = t1 - t0;
  g_rel_ns[1] = t2 - t1;
  g_rel_ns[2] = t3 - t2;
  g_rel_ns[3] = t4 - t3;
  g_rel_ns[4] = 0;
  a.n = a.total = 0;
  a.base = nullptr;
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
  unsigned long long want = 0, gran = 0, total = 0;
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
    int k = got_line ? sscanf(line, "FDS %llu %llu %llu", &want, &gran, &total) : 0;
    if (k == 2) total = want;
    if (k < 2 || total == 0 || want > total || total > (unsigned long long)kArenaMaxGranules || gran == 0) {
      logf(1, "hbm broker %s refused the grant: %s", path, line);
      goto fail;
    }
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
    int rtv = 0;
    auto ver_f = real_hipRuntimeGetVersion();
    if (!ver_f || ver_f(&rtv) != hipSuccess) rtv = 0;
    bool by_address = rtv > 0 && rtv < 70100000;
    logf(1, "hbm broker: runtime %d: fds imported by %s", rtv, by_address ? "address" : "value");
    void* base = nullptr;
    uint64_t vsize = total * gran;
    uint64_t t_r = mono_ns();
    if (reserve_f(&base, vsize, 0, nullptr, 0) != hipSuccess) goto fail;
    g_take_reserve_ns = mono_ns() - t_r;
    g_take_first = uint64_t(got);
    logf(2, "hbm broker: reserved %p + %llu", base, (unsigned long long)vsize);
    int failed = import_and_map(fds, got, a.h, static_cast<char*>(base), gran, by_address);
    a.n = got;  // (released at a failure: the ones imported)
    for (int i = 0; i < got; ++i)
      if (a.h[i]) {
        close(fds[i]);
        fds[i] = -1;
      }
    if (failed) {
      logf(1, "hbm broker: import/map of granule %d failed", failed - 1);
      goto fail;  // the process keeps what it mapped until exit; the broker reclaims at close
    }
    logf(2, "hbm broker: %d granules imported and mapped", got);
    uint64_t t_a = mono_ns();
    if (got && !set_rw(static_cast<char*>(base), uint64_t(got) * gran, dev)) goto fail;
    g_take_access_ns = mono_ns() - t_a;
    a.base = static_cast<char*>(base);
    a.size = a.vsize = vsize;
    a.gran = gran;
    a.total = int(total);
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
  a.live = static_cast<Live*>(calloc(kArenaLiveCap, sizeof(Live)));
  if (!a.ext || !a.live) goto fail;
  a.ext[0] = {0, uint64_t(a.n) * a.gran};
  a.next = a.n ? 1 : 0;
  a.sock = s;
  g_take_connect_ns = t_conn - t_start;
  g_take_wait_ns = t_fds - t_conn;
  g_take_map_ns = mono_ns() - t_fds;
  a.state.store(1, std::memory_order_release);  // base/size published before the state
  logf(1, "hbm broker: %d of %d granules of %llu bytes mapped at %p", a.n, a.total, gran, a.base);
  return;
fail:
  for (int i = 0; i < got; ++i)
    if (fds[i] >= 0) close(fds[i]);
  if (s >= 0) close(s);
}

uint64_t live_slot(uint64_t off) { return (off * 0x9E3779B97F4A7C15ull >> 20) & (kArenaLiveCap - 1); }

bool live_put(uint64_t off, uint64_t len) {
  Arena& a = g_arena;
  if (a.nlive * 2 >= kArenaLiveCap) return false;
  for (uint64_t i = live_slot(off);; i = (i + 1) & (kArenaLiveCap - 1))
    if (!a.live[i].off1) {
      a.live[i] = {off + 1, len, false};
      ++a.nlive;
      return true;
    }
}

bool live_take(uint64_t off, uint64_t* len) {
  Arena& a = g_arena;
  for (uint64_t i = live_slot(off);; i = (i + 1) & (kArenaLiveCap - 1)) {
    Live& l = a.live[i];
    if (!l.off1 && !l.tomb) return false;
    if (l.off1 == off + 1) {
      *len = l.len;
      l.off1 = 0;
      l.tomb = true;
      --a.nlive;
      return true;
    }
  }
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

// first fit; large blocks on 2 MiB boundaries (the CDNA4 TLB fragment), small ones on 4 KiB
bool arena_alloc(uint64_t size, void** ptr) {
  Arena& a = g_arena;
  uint64_t align = size >= (2ull << 20) ? (2ull << 20) : 4096;
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

// [off, off + len) is free again: into the sorted extent list, joined with its neighbours
void ext_insert(uint64_t off, uint64_t len) {
  Arena& a = g_arena;
  int lo = 0, hi = a.next;  // first extent after off
  while (lo < hi) {
    int mid = (lo + hi) / 2;
    if (a.ext[mid].off < off) lo = mid + 1;
    else hi = mid;
  }
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

void arena_free(uint64_t off) {
  Arena& a = g_arena;
  uint64_t len = 0;
  if (!live_take(off, &len)) return;
  a.used -= len;
  ext_insert(off, len);
}

// ---- streaming TAKE: granules owed by the broker ----
// The broker sends "MORE <k> <gran>" and k fds as granules come back (a retiring pod's, once its
// process is gone and they are scrubbed). Each batch is mapped after the granules already there
// and joins the free list. g_arena.mu held.

// the broker will send no more (it went away, or sent something else): the grant shrinks to what
// was delivered, and the ledger with it
void arena_stream_end(const char* why) {
  Arena& a = g_arena;
  logf(1, "hbm broker: stream ended (%s) at %d of %d granules", why, a.n, a.total);
  uint64_t owed = uint64_t(a.total - a.n) * a.gran;
  a.total = a.n;
  a.size -= owed;
  if (a.charged) uncharge(owed);
}

// receive one batch if it arrives within `wait_ms` (0: only one already there); true if the
// arena grew
bool arena_more_locked(int wait_ms) {
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
  if (!recv_line(a.sock, line, sizeof line) || sscanf(line, "MORE %llu %llu", &k, &gran) != 2 || gran != a.gran ||
      k == 0 || k > (unsigned long long)(a.total - a.n)) {
    arena_stream_end(line[0] ? line : "connection closed");
    return false;
  }
  uint64_t t1 = mono_ns();
  int fds[kArenaMaxGranules];
  int got = 0;
  while (got < int(k))
    if (!recv_fd_batch(a.sock, fds, &got, int(k))) {
      for (int i = 0; i < got; ++i) close(fds[i]);
      arena_stream_end("fds lost");
      return false;
    }
  Depth d;
  char* at = a.base + uint64_t(a.n) * a.gran;
  int failed = import_and_map(fds, got, a.h + a.n, at, a.gran, a.by_address);
  for (int i = 0; i < got; ++i) close(fds[i]);
  if (failed || !set_rw(at, uint64_t(got) * a.gran, g_dev)) {
    // keep none of this batch: what was mapped goes, the handles are released
    auto un = real_hipMemUnmap();
    auto rel = real_hipMemRelease();
    for (int i = 0; i < got; ++i)
      if (a.h[a.n + i]) {
        if (un) (void)un(at + uint64_t(i) * a.gran, a.gran);
        if (rel) (void)rel(a.h[a.n + i]);
        a.h[a.n + i] = nullptr;
      }
    arena_stream_end("import/map failed");
    return false;
  }
  ext_insert(uint64_t(a.n) * a.gran, uint64_t(got) * a.gran);
  a.n += got;
  ++g_more_msgs;
  g_more_map_ns += mono_ns() - t1;
  logf(2, "hbm broker: %d more granules, %d of %d mapped", got, a.n, a.total);
  return true;
}

// an allocation of `need` bytes found no room: while the grant has granules still owed that
// would make room, wait for them (GPUSHARE_HBM_MORE_WAIT_S, default 60 s); false: none came
bool arena_wait_more(uint64_t need) {
  Arena& a = g_arena;
  if (a.n >= a.total || need > a.size - a.used) return false;
  static double limit_s = -1;
  if (limit_s < 0) {
    const char* w = getenv("GPUSHARE_HBM_MORE_WAIT_S");
    limit_s = w ? atof(w) : 60.0;
  }
  ++g_more_waits;
  uint64_t deadline = mono_ns() + uint64_t(limit_s * 1e9);
  while (a.n < a.total) {
    if (arena_more_locked(100)) return true;
    if (mono_ns() > deadline) {
      logf(1, "hbm broker: %d granules still owed after %.0f s", a.total - a.n, limit_s);
      return false;
    }
  }
  return false;
}

// ---- stream-ordered frees (hipFreeAsync of arena blocks) ----
// The block goes back to the free list once an event recorded on the freeing stream has
// completed: the kernels that still use it were queued before the event.
struct AsyncFree {
  uint64_t off;
  hipEvent_t ev;
};
constexpr int kMaxAsyncFree = 8192;
AsyncFree g_afree[kMaxAsyncFree];
int g_nafree = 0;  // g_arena.mu held

// return completed stream-ordered frees to the free list (g_arena.mu held); `wait`: all of them
void reap_async_frees(bool wait) {
  auto query = real_hipEventQuery();
  auto sync = real_hipEventSynchronize();
  auto destroy = real_hipEventDestroy();
  Depth d;
  for (int i = 0; i < g_nafree;) {
    hipError_t q = hipSuccess;
    if (g_afree[i].ev) {
      q = wait ? (sync ? sync(g_afree[i].ev) : hipSuccess) : (query ? query(g_afree[i].ev) : hipSuccess);
      if (q == hipErrorNotReady) {
        ++i;
        continue;
      }
      if (destroy) (void)destroy(g_afree[i].ev);
    }
    arena_free(g_afree[i].off);
    g_afree[i] = g_afree[--g_nafree];
  }
}

// 1: served from the arena (*e set), 0: not the arena's (pass through)
int arena_try_alloc(void** ptr, size_t size, hipError_t* e) {
  if (!arena_configured() || size == 0 || t_depth) return 0;
  Arena& a = g_arena;
  pthread_mutex_lock(&a.mu);
  if (a.state == 0) arena_take();
  if (a.state != 1) {
    pthread_mutex_unlock(&a.mu);
    return 0;
  }
  if (g_nafree) reap_async_frees(false);
  while (a.n < a.total && arena_more_locked(0)) {
  }  // owed granules that have arrived
  bool ok = arena_alloc(size, ptr);
  if (!ok && g_nafree) {  // room that stream-ordered frees will give back: wait for them
    reap_async_frees(true);
    ok = arena_alloc(size, ptr);
  }
  while (!ok && arena_wait_more(size)) ok = arena_alloc(size, ptr);  // room the broker still owes
  pthread_mutex_unlock(&a.mu);
  if (!ok) {
    if (ptr) *ptr = nullptr;
    logf(1, "hbm broker arena: deny %zu bytes (used %llu of %llu)", size, (unsigned long long)a.used,
         (unsigned long long)a.size);
    *e = hipErrorOutOfMemory;
  } else {
    *e = hipSuccess;
  }
  return 1;
}

bool arena_owns(void* p) {
  Arena& a = g_arena;
  return a.state.load(std::memory_order_acquire) == 1 && static_cast<char*>(p) >= a.base &&
         static_cast<char*>(p) < a.base + a.size;
}

// ---- VMM from the arena (PyTorch's expandable segments) ----------------------------------------
// A VMM user reserves a large VA range (hipMemAddressReserve), creates small physical handles
// (hipMemCreate, 2 / 20 MiB pages for PyTorch) and maps them one after another into the range.
// Physical handles of the arena cannot be cut into pages, so the shim lends whole granules:
// a reservation of >= 1 GiB (a "window") is aligned to the granule, its granule-sized slots are
// backed on demand by arena granules (unmapped from the arena's own range and mapped into the
// slot), and the user's handles are stand-ins whose map is a no-op inside a backed slot. A slot
// whose pages are all unmapped gives its granule back to the arena. When no granule is free, the
// slot is served by real handles from the driver (charged to the quota as before).
constexpr uint64_t kWinAlign = 1ull << 30;
constexpr int kMaxWin = 64;
constexpr uint64_t kVHandleMagic = 0x67737668616e646cull;  // "gsvhandl"

struct Win {
  char* base;
  uint64_t size;
  char* vbase;     // the reservation it lies in (larger when the runtime ignored the alignment)
  uint64_t vsize;
  int nslots;
  int32_t* slot_g;      // arena granule backing the slot, -1 none
  uint64_t* slot_used;  // bytes of stand-in pages mapped in the slot (arena-backed slots)
  uint32_t* slot_real;  // real (driver) pieces mapped in the slot
};
Win g_win[kMaxWin];
int g_nwin = 0;

struct VPiece {
  char* va;
  uint64_t len;
  hipMemGenericAllocationHandle_t h;  // real handle (driver), or nullptr: inside an arena slot
};
struct VHandle {
  uint64_t magic;
  uint64_t size;
  hipMemAllocationProp prop;
  unsigned long long flags;
  char* at;  // mapped at (nullptr: not mapped)
  int npieces;
  VPiece* pieces;
};

// stand-in handles and their mapped addresses: open addressing on the pointer / VA
constexpr uint64_t kVCap = 1 << 17;
uintptr_t* g_vh = nullptr;   // VHandle* set
uintptr_t* g_vva = nullptr;  // VA -> VHandle* (pairs)
uint64_t g_vh_n = 0, g_vva_n = 0, g_pending_bytes = 0;
uint64_t g_vmm_arena_maps = 0, g_vmm_real_pieces = 0, g_vmm_creates = 0, g_slots_backed = 0, g_vmm_span_access = 0;

bool vtables() {
  if (!g_vh) g_vh = static_cast<uintptr_t*>(calloc(kVCap, sizeof(uintptr_t)));
  if (!g_vva) g_vva = static_cast<uintptr_t*>(calloc(2 * kVCap, sizeof(uintptr_t)));
  return g_vh && g_vva;
}
uint64_t vslot(uintptr_t k) { return (k * 0x9E3779B97F4A7C15ull >> 17) & (kVCap - 1); }
constexpr uintptr_t kTomb = ~uintptr_t(0);

bool vh_put(VHandle* h) {
  if (g_vh_n * 2 >= kVCap) return false;
  uintptr_t k = reinterpret_cast<uintptr_t>(h);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1))
    if (!g_vh[i] || g_vh[i] == kTomb) {
      g_vh[i] = k;
      ++g_vh_n;
      return true;
    }
}
bool vh_has(const void* p) {
  if (!g_vh || !p) return false;
  uintptr_t k = reinterpret_cast<uintptr_t>(p);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1)) {
    if (!g_vh[i]) return false;
    if (g_vh[i] == k) return true;
  }
}
void vh_del(VHandle* h) {
  uintptr_t k = reinterpret_cast<uintptr_t>(h);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1)) {
    if (!g_vh[i]) return;
    if (g_vh[i] == k) {
      g_vh[i] = kTomb;
      --g_vh_n;
      return;
    }
  }
}
bool vva_put(char* va, VHandle* h) {
  if (g_vva_n * 2 >= kVCap) return false;
  uintptr_t k = reinterpret_cast<uintptr_t>(va);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1))
    if (!g_vva[2 * i] || g_vva[2 * i] == kTomb) {
      g_vva[2 * i] = k;
      g_vva[2 * i + 1] = reinterpret_cast<uintptr_t>(h);
      ++g_vva_n;
      return true;
    }
}
VHandle* vva_take(char* va) {
  if (!g_vva) return nullptr;
  uintptr_t k = reinterpret_cast<uintptr_t>(va);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1)) {
    if (!g_vva[2 * i]) return nullptr;
    if (g_vva[2 * i] == k) {
      g_vva[2 * i] = kTomb;
      --g_vva_n;
      return reinterpret_cast<VHandle*>(g_vva[2 * i + 1]);
    }
  }
}

// where the run of mappings that ends at `at` without a hole begins, in window `w`: whole arena
// slots and the driver pieces mapped in the other slots (g_arena.mu held)
struct Span {
  char* va;
  uint64_t len;
};
int span_cmp(const void* x, const void* y) {
  const char* a = static_cast<const Span*>(x)->va;
  const char* b = static_cast<const Span*>(y)->va;
  return a < b ? -1 : a > b;
}
char* mapped_run_start(Win& w, char* at) {
  uint64_t cap = 256, n = 0;
  Span* v = static_cast<Span*>(malloc(cap * sizeof(Span)));
  for (uint64_t i = 0; v && g_vva && i < kVCap; ++i) {
    uintptr_t k = g_vva[2 * i];
    if (!k || k == kTomb) continue;
    VHandle* h = reinterpret_cast<VHandle*>(g_vva[2 * i + 1]);
    for (int j = 0; j < h->npieces; ++j) {
      VPiece& pc = h->pieces[j];
      if (!pc.h || pc.va < w.base || pc.va >= w.base + w.size) continue;
      if (n == cap) {
        Span* g = static_cast<Span*>(realloc(v, 2 * cap * sizeof(Span)));
        if (!g) break;
        v = g;
        cap *= 2;
      }
      v[n++] = {pc.va, pc.len};
    }
  }
  if (v) qsort(v, n, sizeof(Span), span_cmp);
  char* cur = at;
  while (v && cur > w.base) {
    int s = int(uint64_t(cur - 1 - w.base) / kWinAlign);
    char* st = w.base + uint64_t(s) * kWinAlign;
    if (w.slot_g[s] >= 0) {  // an arena slot: one mapping of its whole granule
      if (cur != st + kWinAlign) break;
      cur = st;
      continue;
    }
    uint64_t lo = 0, hi = n;  // the last driver piece starting below cur
    while (lo < hi) {
      uint64_t mid = (lo + hi) / 2;
      if (v[mid].va < cur) lo = mid + 1;
      else hi = mid;
    }
    if (lo == 0 || v[lo - 1].va + v[lo - 1].len != cur) break;
    cur = v[lo - 1].va;
  }
  free(v);
  return cur;
}


Win* win_of(const char* p, uint64_t len) {
  for (int i = 0; i < g_nwin; ++i)
    if (p >= g_win[i].base && p + len <= g_win[i].base + g_win[i].size) return &g_win[i];
  return nullptr;
}

// back slot s of window w with an arena granule (g_arena.mu held); false: none free (or the
// broker's granule is not the slot size: then every page is the driver's)
bool slot_back(Win& w, int s) {
  Arena& a = g_arena;
  uint64_t off;
  if (a.state.load(std::memory_order_relaxed) != 1 || a.gran != kWinAlign) return false;
  while (a.n < a.total && arena_more_locked(0)) {
  }
  bool got = arena_take_granule(&off);
  while (!got && arena_wait_more(a.gran)) got = arena_take_granule(&off);
  if (!got) return false;
  int gi = int(off / a.gran);
  auto un = real_hipMemUnmap();
  auto map = real_hipMemMap();
  char* slot = w.base + uint64_t(s) * kWinAlign;
  Depth d;
  if (!un || !map || un(a.base + off, a.gran) != hipSuccess) {
    arena_free(off);
    return false;
  }
  if (map(slot, a.gran, 0, a.h[gi], 0) != hipSuccess || !set_rw(slot, a.gran, g_dev)) {
    // back where it was: the arena's own range keeps every granule it does not lend
    if (map(a.base + off, a.gran, 0, a.h[gi], 0) == hipSuccess) set_rw(a.base + off, a.gran, g_dev);
    arena_free(off);
    return false;
  }
  w.slot_g[s] = gi;
  w.slot_used[s] = 0;
  ++g_slots_backed;
  return true;
}

// the slot's last page is gone: its granule goes back to the arena (g_arena.mu held)
void slot_return(Win& w, int s) {
  Arena& a = g_arena;
  int gi = w.slot_g[s];
  if (gi < 0) return;
  auto un = real_hipMemUnmap();
  auto map = real_hipMemMap();
  char* slot = w.base + uint64_t(s) * kWinAlign;
  Depth d;
  if (auto sync = real_hipDeviceSynchronize()) (void)sync();   // nothing may still use it when it moves
  if (un) (void)un(slot, a.gran);
  if (map && map(a.base + uint64_t(gi) * a.gran, a.gran, 0, a.h[gi], 0) == hipSuccess)
    set_rw(a.base + uint64_t(gi) * a.gran, a.gran, g_dev);
  arena_free(uint64_t(gi) * a.gran);
  w.slot_g[s] = -1;
  w.slot_used[s] = 0;
}

// bytes a new stand-in handle could still be given: free arena granules, unmapped room in the
// backed slots, less what stand-ins created but not mapped yet will take (g_arena.mu held)
uint64_t vmm_room() {
  Arena& a = g_arena;
  uint64_t room = a.size - a.used;
  for (int i = 0; i < g_nwin; ++i)
    for (int s = 0; s < g_win[i].nslots; ++s)
      if (g_win[i].slot_g[s] >= 0) room += kWinAlign - g_win[i].slot_used[s];
  return room > g_pending_bytes ? room - g_pending_bytes : 0;
}

hipError_t real_create_charged(hipMemGenericAllocationHandle_t* h, size_t size, const hipMemAllocationProp* prop,
                               unsigned long long flags);

// map stand-in `v` at [va, va + v->size) inside window `w` (g_arena.mu held)
hipError_t vmm_map(Win& w, VHandle* v, char* va) {
  uint64_t lo = uint64_t(va - w.base), hi = lo + v->size;
  int s0 = int(lo / kWinAlign), s1 = int((hi - 1) / kWinAlign);
  v->pieces = static_cast<VPiece*>(calloc(size_t(s1 - s0 + 1), sizeof(VPiece)));
  if (!v->pieces) return hipErrorOutOfMemory;
  v->npieces = 0;
  v->at = va;  // (vmm_unmap undoes a partial map)
  auto map = real_hipMemMap();
  for (int s = s0; s <= s1; ++s) {
    uint64_t plo = s == s0 ? lo : uint64_t(s) * kWinAlign;
    uint64_t phi = s == s1 ? hi : uint64_t(s + 1) * kWinAlign;
    VPiece& pc = v->pieces[v->npieces];
    pc.va = w.base + plo;
    pc.len = phi - plo;
    pc.h = nullptr;
    if (w.slot_g[s] < 0 && w.slot_real[s] == 0) slot_back(w, s);
    if (w.slot_g[s] >= 0) {
      w.slot_used[s] += pc.len;
      ++g_vmm_arena_maps;
    } else {
      // the driver: a real handle of this piece's size, mapped in the slot (charged as any other)
      hipError_t e = real_create_charged(&pc.h, pc.len, &v->prop, v->flags);
      if (e == hipSuccess) {
        Depth d;
        e = map ? map(pc.va, pc.len, 0, pc.h, 0) : hipErrorNotInitialized;
        if (e != hipSuccess) hipMemRelease(pc.h);
      }
      if (e != hipSuccess) {
        logf(1, "vmm: driver piece of %llu bytes at slot %d + %llu: error %d", (unsigned long long)pc.len, s,
             (unsigned long long)(plo - uint64_t(s) * kWinAlign), int(e));
        return e;  // the caller undoes the pieces mapped so far
      }
      ++w.slot_real[s];
      ++g_vmm_real_pieces;
      logf(2, "vmm: driver piece of %llu bytes mapped at +%llu", (unsigned long long)pc.len, (unsigned long long)plo);
    }
    ++v->npieces;
  }
  return hipSuccess;
}

// unmap stand-in `v` (g_arena.mu held); its real pieces are released with it (hipMemRelease)
void vmm_unmap(VHandle* v) {
  Win* w = v->at ? win_of(v->at, v->size) : nullptr;
  auto un = real_hipMemUnmap();
  for (int i = 0; i < v->npieces && w; ++i) {
    VPiece& pc = v->pieces[i];
    int s = int(uint64_t(pc.va - w->base) / kWinAlign);
    if (pc.h) {
      Depth d;
      if (un) (void)un(pc.va, pc.len);
      --w->slot_real[s];
    } else if (w->slot_g[s] >= 0) {
      w->slot_used[s] -= pc.len;
      if (w->slot_used[s] == 0) slot_return(*w, s);
    }
  }
  v->at = nullptr;
}

void vmm_release_pieces(VHandle* v) {
  for (int i = 0; i < v->npieces; ++i)
    if (v->pieces[i].h) hipMemRelease(v->pieces[i].h);   // the interposed release: uncharged
  free(v->pieces);
  v->pieces = nullptr;
  v->npieces = 0;
}
}  // namespace

// ---- interposed HIP API --------------------------------------------------------------------
GS_EXPORT hipError_t hipMalloc(void** ptr, size_t size) {
  auto f = real_hipMalloc();
  if (!f) return hipErrorNotInitialized;
  hipError_t ae;
  if (arena_try_alloc(ptr, size, &ae)) return ae;
  return guarded_alloc(ptr, size, [&] { return f(ptr, size); });
}

// Hand the arena back to the broker now (the pod is retiring and freed everything). Returns 1 if
// released, 0 if there is no arena, -1 if allocations are still live in it.
GS_EXPORT int gpushare_shim_arena_release() {
  Arena& a = g_arena;
  pthread_mutex_lock(&a.mu);
  if (a.state != 1) {
    pthread_mutex_unlock(&a.mu);
    return 0;
  }
  if (g_nafree) reap_async_frees(true);
  if (a.nlive) {  // (granules lent to VMM windows are live blocks too)
    pthread_mutex_unlock(&a.mu);
    return -1;
  }
  arena_unmap_locked();
  if (a.rt_version > 0 && a.rt_version < 70100000 && env_u64("GPUSHARE_HBM_FREE_KEPT", 1)) {
    // HIP 7.0 keeps the KFD imports of the released handles: free them, so the broker sees its
    // granules' references gone now rather than at this process's teardown
    uint64_t t = mono_ns();
    int n = imports_free_kept(real_ioctl());
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

// VMM from the arena: stand-ins created, pages mapped into arena slots, driver pieces, slots backed
// by a granule so far, and granules lent to windows now
GS_EXPORT int gpushare_shim_vmm_stats(uint64_t* creates, uint64_t* arena_maps, uint64_t* real_pieces,
                                      uint64_t* slots_backed, uint64_t* slots_now) {
  pthread_mutex_lock(&g_arena.mu);
  uint64_t now = 0;
  for (int i = 0; i < g_nwin; ++i)
    for (int sl = 0; sl < g_win[i].nslots; ++sl) now += g_win[i].slot_g[sl] >= 0;
  if (creates) *creates = g_vmm_creates;
  if (arena_maps) *arena_maps = g_vmm_arena_maps;
  if (real_pieces) *real_pieces = g_vmm_real_pieces;
  if (slots_backed) *slots_backed = g_slots_backed;
  if (slots_now) *slots_now = now;
  int n = g_nwin;
  pthread_mutex_unlock(&g_arena.mu);
  return n;
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

// the process's first granule import and map (ns): the runtime's one-time work inside the TAKE;
// and how long the TAKE waited for the broker's answer line
GS_EXPORT int gpushare_shim_arena_first(uint64_t* import_ns, uint64_t* map_ns, uint64_t* header_ns) {
  if (import_ns) *import_ns = g_first_import_ns;
  if (map_ns) *map_ns = g_first_map_ns;
  if (header_ns) *header_ns = g_take_header_ns;
  return g_first_import_ns != 0;
}

// (size, used) of the arena; 0 when there is none
GS_EXPORT int gpushare_shim_arena_stats(uint64_t* size, uint64_t* used) {
  Arena& a = g_arena;
  pthread_mutex_lock(&a.mu);
  int on = a.state == 1;
  if (size) *size = on ? a.size : 0;
  if (used) *used = on ? a.used : 0;
  pthread_mutex_unlock(&a.mu);
  return on;
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

namespace {
// a stream under graph capture records its allocations into the graph: those stay the driver's
bool capturing(hipStream_t stream) {
  auto f = real_hipStreamIsCapturing();
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  Depth d;
  return f && f(stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}
}  // namespace

// Stream-ordered allocations (PyTorch's cudaMallocAsync backend) come from the arena too: the
// memory is there at once, and a stream-ordered free returns it once the stream got past it.
GS_EXPORT hipError_t hipMallocAsync(void** ptr, size_t size, hipStream_t stream) {
  auto f = real_hipMallocAsync();
  if (!f) return hipErrorNotInitialized;
  hipError_t ae;
  if (arena_configured() && !capturing(stream) && arena_try_alloc(ptr, size, &ae)) return ae;
  return guarded_alloc(ptr, size, [&] { return f(ptr, size, stream); });
}

// from the device's default pool only: a pool the program made has attributes of its own
// (IPC export, a release threshold it watches) that the arena does not give
GS_EXPORT hipError_t hipMallocFromPoolAsync(void** ptr, size_t size, hipMemPool_t pool, hipStream_t stream) {
  auto f = real_hipMallocFromPoolAsync();
  if (!f) return hipErrorNotInitialized;
  if (arena_configured() && !capturing(stream)) {
    hipMemPool_t dflt = nullptr;
    int dev = 0;
    auto gd = real_hipGetDevice();
    auto dp = real_hipDeviceGetDefaultMemPool();
    bool is_default;
    {
      Depth d;
      is_default = gd && dp && gd(&dev) == hipSuccess && dp(&dflt, dev) == hipSuccess && dflt == pool;
    }
    hipError_t ae;
    if (is_default && arena_try_alloc(ptr, size, &ae)) return ae;
  }
  return guarded_alloc(ptr, size, [&] { return f(ptr, size, pool, stream); });
}

GS_EXPORT hipError_t hipMallocPitch(void** ptr, size_t* pitch, size_t width, size_t height) {
  auto f = real_hipMallocPitch();
  if (!f) return hipErrorNotInitialized;
  if (!hip_active()) return f(ptr, pitch, width, height);
  hipError_t e;
  {
    Depth d;
    e = f(ptr, pitch, width, height);
  }
  if (e != hipSuccess || !ptr || !*ptr) return e;
  uint64_t c = charge_of(*pitch * height);
  if (!charge(c)) {
    Depth d;
    if (auto fr = real_hipFree()) (void)fr(*ptr);
    *ptr = nullptr;
    return deny(*pitch * height);
  }
  track((uint64_t)(uintptr_t)*ptr, c);
  return e;
}

GS_EXPORT hipError_t hipMalloc3D(hipPitchedPtr* pp, hipExtent ext) {
  auto f = real_hipMalloc3D();
  if (!f) return hipErrorNotInitialized;
  if (!hip_active()) return f(pp, ext);
  hipError_t e;
  {
    Depth d;
    e = f(pp, ext);
  }
  if (e != hipSuccess || !pp || !pp->ptr) return e;
  uint64_t c = charge_of(pp->pitch * ext.height * ext.depth);
  if (!charge(c)) {
    Depth d;
    if (auto fr = real_hipFree()) (void)fr(pp->ptr);
    pp->ptr = nullptr;
    return deny(pp->pitch * ext.height * ext.depth);
  }
  track((uint64_t)(uintptr_t)pp->ptr, c);
  return e;
}

GS_EXPORT hipError_t hipFree(void* ptr) {
  auto f = real_hipFree();
  if (!f) return hipErrorNotInitialized;
  if (ptr && arena_configured() && arena_owns(ptr)) {
    // the caching allocator frees after its streams' work; a plain hipFree synchronises the
    // device first, so do the same before the range can be handed out again
    Depth d;
    if (auto dev_sync = real_hipDeviceSynchronize()) (void)dev_sync();
    pthread_mutex_lock(&g_arena.mu);
    arena_free(uint64_t(static_cast<char*>(ptr) - g_arena.base));
    pthread_mutex_unlock(&g_arena.mu);
    return hipSuccess;
  }
  if (!hip_active() || !ptr) return f(ptr);
  hipError_t e;
  {
    Depth d;
    e = f(ptr);
  }
  if (e == hipSuccess) uncharge(untrack((uint64_t)(uintptr_t)ptr));
  return e;
}

GS_EXPORT hipError_t hipFreeAsync(void* ptr, hipStream_t stream) {
  auto f = real_hipFreeAsync();
  if (!f) return hipErrorNotInitialized;
  if (ptr && arena_configured() && arena_owns(ptr)) {
    uint64_t off = uint64_t(static_cast<char*>(ptr) - g_arena.base);
    hipEvent_t ev = nullptr;
    auto mk = real_hipEventCreateWithFlags();
    auto rec = real_hipEventRecord();
    bool ok;
    {
      Depth d;
      ok = mk && rec && mk(&ev, hipEventDisableTiming) == hipSuccess;
      if (ok && rec(ev, stream) != hipSuccess) {
        if (auto de = real_hipEventDestroy()) (void)de(ev);
        ok = false;
      }
      if (!ok) {  // no event: wait for the device instead, as a plain hipFree does
        ev = nullptr;
        if (auto dev_sync = real_hipDeviceSynchronize()) (void)dev_sync();
      }
    }
    pthread_mutex_lock(&g_arena.mu);
    if (g_nafree == kMaxAsyncFree) reap_async_frees(true);
    g_afree[g_nafree++] = {off, ev};
    pthread_mutex_unlock(&g_arena.mu);
    return hipSuccess;
  }
  if (!hip_active() || !ptr) return f(ptr, stream);
  hipError_t e;
  {
    Depth d;
    e = f(ptr, stream);
  }
  if (e == hipSuccess) uncharge(untrack((uint64_t)(uintptr_t)ptr));
  return e;
}

namespace {
// the driver's hipMemCreate under the quota (hip mode charges here; kfd mode at the ioctl)
hipError_t real_create_charged(hipMemGenericAllocationHandle_t* handle, size_t size, const hipMemAllocationProp* prop,
                               unsigned long long flags) {
  auto f = real_hipMemCreate();
  if (!f) return hipErrorNotInitialized;
  if (!hip_active()) {
    Depth d;
    return f(handle, size, prop, flags);
  }
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
  track((uint64_t)(uintptr_t)*handle, c);
  return e;
}

// with a broker arena: VMM on the device is served from it (see "VMM from the arena")
bool vmm_from_arena(const hipMemAllocationProp* prop) {
  if (!arena_configured() || t_depth || !prop || prop->type != hipMemAllocationTypePinned ||
      prop->location.type != hipMemLocationTypeDevice)
    return false;
  Arena& a = g_arena;
  if (a.state.load(std::memory_order_acquire) == 0) {
    pthread_mutex_lock(&a.mu);
    if (a.state == 0) arena_take();
    pthread_mutex_unlock(&a.mu);
  }
  return a.state.load(std::memory_order_acquire) == 1 && prop->location.id == g_dev;
}
}  // namespace

GS_EXPORT hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* handle, size_t size,
                                  const hipMemAllocationProp* prop, unsigned long long flags) {
  if (!real_hipMemCreate()) return hipErrorNotInitialized;
  if (handle && size && vmm_from_arena(prop)) {
    // a stand-in: its memory is decided where it is mapped (an arena slot, or the driver)
    Arena& a = g_arena;
    pthread_mutex_lock(&a.mu);
    bool ok = vtables();
    if (ok) {
      uint64_t left = 0, quota = g.quota.load();
      if (enabled() && quota) {
        uint64_t used = g.ledger->total.load();
        left = used >= quota ? 0 : quota - used;
      }
      ok = vmm_room() + left >= size;
    }
    VHandle* v = ok ? static_cast<VHandle*>(calloc(1, sizeof(VHandle))) : nullptr;
    if (v) {
      v->magic = kVHandleMagic;
      v->size = size;
      v->prop = *prop;
      v->flags = flags;
      if (!vh_put(v)) {
        free(v);
        v = nullptr;
      }
    }
    if (v) {
      g_pending_bytes += size;
      ++g_vmm_creates;
    }
    pthread_mutex_unlock(&a.mu);
    if (!v) {
      logf(1, "vmm: deny a handle of %zu bytes (arena and quota full)", size);
      return hipErrorOutOfMemory;  // what the driver says when memory is out: callers handle it
    }
    *handle = reinterpret_cast<hipMemGenericAllocationHandle_t>(v);
    return hipSuccess;
  }
  return real_create_charged(handle, size, prop, flags);
}

GS_EXPORT hipError_t hipMemAddressReserve(void** ptr, size_t size, size_t alignment, void* addr,
                                          unsigned long long flags) {
  auto f = real_hipMemAddressReserve();
  if (!f) return hipErrorNotInitialized;
  bool window = arena_configured() && !t_depth && size >= kWinAlign && !addr;
  if (window && alignment < kWinAlign) alignment = kWinAlign;  // slots on granule boundaries
  hipError_t e;
  char* vbase = nullptr;
  uint64_t vsize = size;
  {
    Depth d;
    e = f(ptr, size, alignment, addr, flags);
    vbase = e == hipSuccess && ptr ? static_cast<char*>(*ptr) : nullptr;
    if (window && vbase && reinterpret_cast<uintptr_t>(vbase) % kWinAlign) {
      // the runtime does not honour so large an alignment (HIP 7.x returns a 2 MiB-aligned range):
      // reserve one granule more and use its aligned part; the whole reservation is freed with it
      (void)real_hipMemAddressFree()(vbase, size);
      void* big = nullptr;
      if (f(&big, size + kWinAlign, 0, nullptr, flags) == hipSuccess && big) {
        vbase = static_cast<char*>(big);
        vsize = size + kWinAlign;
        *ptr = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(big) + kWinAlign - 1) & ~uintptr_t(kWinAlign - 1));
      } else {
        window = false;  // no aligned range: an ordinary reservation, its pages from the driver
        e = f(ptr, size, 0, addr, flags);
        vbase = nullptr;
      }
    }
  }
  if (e != hipSuccess || !window || !ptr || !*ptr) return e;
  pthread_mutex_lock(&g_arena.mu);
  if (g_nwin < kMaxWin) {
    Win& w = g_win[g_nwin];
    w.base = static_cast<char*>(*ptr);
    w.size = size;
    w.vbase = vbase;
    w.vsize = vsize;
    w.nslots = int((size + kWinAlign - 1) / kWinAlign);
    w.slot_g = static_cast<int32_t*>(malloc(sizeof(int32_t) * size_t(w.nslots)));
    w.slot_used = static_cast<uint64_t*>(calloc(size_t(w.nslots), sizeof(uint64_t)));
    w.slot_real = static_cast<uint32_t*>(calloc(size_t(w.nslots), sizeof(uint32_t)));
    if (w.slot_g && w.slot_used && w.slot_real) {
      for (int i = 0; i < w.nslots; ++i) w.slot_g[i] = -1;
      ++g_nwin;
    } else {
      free(w.slot_g), free(w.slot_used), free(w.slot_real);
    }
  }
  pthread_mutex_unlock(&g_arena.mu);
  return e;
}

GS_EXPORT hipError_t hipMemAddressFree(void* ptr, size_t size) {
  auto f = real_hipMemAddressFree();
  if (!f) return hipErrorNotInitialized;
  char* vbase = static_cast<char*>(ptr);
  uint64_t vsize = size;
  if (ptr && arena_configured() && !t_depth) {
    pthread_mutex_lock(&g_arena.mu);
    for (int i = 0; i < g_nwin; ++i) {
      if (g_win[i].base != ptr) continue;
      Win& w = g_win[i];
      for (int sl = 0; sl < w.nslots; ++sl)
        if (w.slot_g[sl] >= 0) slot_return(w, sl);   // pages the program never unmapped
      free(w.slot_g), free(w.slot_used), free(w.slot_real);
      vbase = w.vbase;
      vsize = w.vsize;
      g_win[i] = g_win[--g_nwin];
      break;
    }
    pthread_mutex_unlock(&g_arena.mu);
  }
  Depth d;
  return f(vbase, vsize);
}

GS_EXPORT hipError_t hipMemMap(void* ptr, size_t size, size_t offset, hipMemGenericAllocationHandle_t handle,
                               unsigned long long flags) {
  auto f = real_hipMemMap();
  if (!f) return hipErrorNotInitialized;
  if (t_depth || !arena_configured()) return f(ptr, size, offset, handle, flags);
  pthread_mutex_lock(&g_arena.mu);
  if (!vh_has(handle)) {
    pthread_mutex_unlock(&g_arena.mu);
    return f(ptr, size, offset, handle, flags);
  }
  VHandle* v = reinterpret_cast<VHandle*>(handle);
  char* va = static_cast<char*>(ptr);
  hipError_t e = hipErrorInvalidValue;
  Win* w = va && !v->at && offset == 0 && size == v->size ? win_of(va, size) : nullptr;
  if (w) {
    e = vmm_map(*w, v, va);
    if (e != hipSuccess) {
      vmm_unmap(v);
      vmm_release_pieces(v);
    } else {
      g_pending_bytes -= v->size;
      vva_put(va, v);
    }
  } else if (va && !v->at && offset == 0 && size == v->size) {
    // outside every window: the driver's memory for it, mapped where asked
    VPiece* pc = static_cast<VPiece*>(calloc(1, sizeof(VPiece)));
    if (pc) {
      e = real_create_charged(&pc->h, size, &v->prop, v->flags);
      if (e == hipSuccess) {
        Depth d;
        e = f(va, size, 0, pc->h, flags);
        if (e != hipSuccess) hipMemRelease(pc->h);
      }
      if (e == hipSuccess) {
        pc->va = va;
        pc->len = size;
        v->pieces = pc;
        v->npieces = 1;
        v->at = va;
        g_pending_bytes -= v->size;
        vva_put(va, v);
        ++g_vmm_real_pieces;
      } else {
        free(pc);
      }
    } else {
      e = hipErrorOutOfMemory;
    }
  }
  pthread_mutex_unlock(&g_arena.mu);
  return e;
}

GS_EXPORT hipError_t hipMemUnmap(void* ptr, size_t size) {
  auto f = real_hipMemUnmap();
  if (!f) return hipErrorNotInitialized;
  if (t_depth || !arena_configured() || !g_vva) return f(ptr, size);
  pthread_mutex_lock(&g_arena.mu);
  // the program unmaps what it mapped, one handle's range at a time (or several at once)
  char* va = static_cast<char*>(ptr);
  char* end = va + size;
  bool any = false;
  while (va < end) {
    VHandle* v = vva_take(va);
    if (!v) break;
    any = true;
    if (win_of(v->at, v->size)) {
      vmm_unmap(v);
    } else {  // the driver piece mapped outside the windows
      Depth d;
      (void)f(v->at, v->size);
      v->at = nullptr;
    }
    va += v->size;
  }
  pthread_mutex_unlock(&g_arena.mu);
  if (any) return va == end ? hipSuccess : f(va, size_t(end - va));
  return f(ptr, size);
}

GS_EXPORT hipError_t hipMemSetAccess(void* ptr, size_t size, const hipMemAccessDesc* desc, size_t count) {
  auto f = real_hipMemSetAccess();
  if (!f) return hipErrorNotInitialized;
  if (t_depth || !arena_configured() || !ptr || !g_nwin) return f(ptr, size, desc, count);
  pthread_mutex_lock(&g_arena.mu);
  Win* w = win_of(static_cast<char*>(ptr), size);
  if (!w) {
    pthread_mutex_unlock(&g_arena.mu);
    return f(ptr, size, desc, count);
  }
  // slot by slot: the driver's memory in the range (real pages, driver pieces) gets the access
  // asked for, run by run; an arena slot is one granule mapping, read-write for this device
  // since it was backed: only access for other devices is set, on the whole granule
  bool local_rw = true;
  for (size_t k = 0; k < count; ++k)
    local_rw = local_rw && desc[k].location.type == hipMemLocationTypeDevice && desc[k].location.id == g_dev &&
               desc[k].flags == hipMemAccessFlagsProtReadWrite;
  char* lo = static_cast<char*>(ptr);
  char* hi = lo + size;
  char* run = nullptr;  // start of the current run of driver memory
  hipError_t e = hipSuccess;
  Depth d;
  auto set = [&](char* at, size_t n) {
    hipError_t r = f(at, n, desc, count);
    logf(2, "vmm: access +%llu, %zu bytes: %d", (unsigned long long)(at - w->base), n, int(r));
    if (r != hipSuccess && local_rw) {
      // HIP 7.x refuses, now and then, the access of a driver page mapped after a mapping of
      // another size in the same range, while one call over the whole run of mappings ending at
      // that page succeeds (tools/diag/vmm_spill_probe.cpp, profiles/r5/vmm_spill_probe_run*.json)
      char* from = mapped_run_start(*w, at);
      if (from < at) {
        if (auto le = real_hipGetLastError()) (void)le();
        r = f(from, size_t(at + n - from), desc, count);
        ++g_vmm_span_access;
        logf(1, "vmm: access of +%llu refused; over the run from +%llu (%llu bytes): %d",
             (unsigned long long)(at - w->base), (unsigned long long)(from - w->base),
             (unsigned long long)(at + n - from), int(r));
      }
    }
    return r;
  };
  for (char* p = lo; p < hi && e == hipSuccess;) {
    int s = int(uint64_t(p - w->base) / kWinAlign);
    char* send = w->base + uint64_t(s + 1) * kWinAlign;
    char* q = send < hi ? send : hi;
    if (w->slot_g[s] >= 0) {
      if (run) e = set(run, size_t(p - run)), run = nullptr;
      if (e == hipSuccess && !local_rw) e = set(w->base + uint64_t(s) * kWinAlign, kWinAlign);
    } else if (!run) {
      run = p;
    }
    p = q;
  }
  if (run && e == hipSuccess) e = set(run, size_t(hi - run));
  if (e != hipSuccess)
    logf(1, "vmm: access for window +%llu, %zu bytes: error %d", (unsigned long long)(lo - w->base), size, int(e));
  pthread_mutex_unlock(&g_arena.mu);
  return e;
}

GS_EXPORT hipError_t hipMemGetAllocationPropertiesFromHandle(hipMemAllocationProp* prop,
                                                             hipMemGenericAllocationHandle_t handle) {
  auto f = real_hipMemGetAllocationPropertiesFromHandle();
  if (!f) return hipErrorNotInitialized;
  if (arena_configured() && g_vh) {
    pthread_mutex_lock(&g_arena.mu);
    bool mine = vh_has(handle);
    if (mine && prop) *prop = reinterpret_cast<VHandle*>(handle)->prop;
    pthread_mutex_unlock(&g_arena.mu);
    if (mine) return prop ? hipSuccess : hipErrorInvalidValue;
  }
  return f(prop, handle);
}

GS_EXPORT hipError_t hipMemExportToShareableHandle(void* out, hipMemGenericAllocationHandle_t handle,
                                                   hipMemAllocationHandleType type, unsigned long long flags) {
  auto f = real_hipMemExportToShareableHandle();
  if (!f) return hipErrorNotInitialized;
  if (arena_configured() && g_vh) {
    pthread_mutex_lock(&g_arena.mu);
    bool mine = vh_has(handle);
    pthread_mutex_unlock(&g_arena.mu);
    // an arena page is part of a granule another pod had and will have: it is never exported
    if (mine) return hipErrorNotSupported;
  }
  return f(out, handle, type, flags);
}

GS_EXPORT hipError_t hipMemRelease(hipMemGenericAllocationHandle_t handle) {
  auto f = real_hipMemRelease();
  if (!f) return hipErrorNotInitialized;
  if (arena_configured() && g_vh) {
    pthread_mutex_lock(&g_arena.mu);
    if (vh_has(handle)) {
      VHandle* v = reinterpret_cast<VHandle*>(handle);
      if (v->at) {  // released while mapped: the mapping goes with it
        char* at = v->at;
        (void)vva_take(at);
        if (win_of(at, v->size)) {
          vmm_unmap(v);
        } else if (auto un = real_hipMemUnmap()) {
          Depth d;
          (void)un(at, v->size);
          v->at = nullptr;
        }
      } else if (!v->npieces) {
        g_pending_bytes -= v->size;
      }
      vh_del(v);
      pthread_mutex_unlock(&g_arena.mu);
      vmm_release_pieces(v);
      v->magic = 0;
      free(v);
      return hipSuccess;
    }
    pthread_mutex_unlock(&g_arena.mu);
  }
  if (!hip_active()) return f(handle);
  hipError_t e;
  {
    Depth d;
    e = f(handle);
  }
  if (e == hipSuccess) uncharge(untrack((uint64_t)(uintptr_t)handle));
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
  if (e != hipSuccess || !enabled() || t_depth) return e;
  if (!g.quota.load() && total_b) set_quota_from_device_bytes(*total_b);
  uint64_t quota = g.quota.load();
  if (!quota) return e;
  uint64_t used = g.ledger->total.load();
  uint64_t left = used >= quota ? 0 : quota - used;
  if (free_b && *free_b > left) *free_b = (size_t)left;
  if (total_b) *total_b = (size_t)quota;
  uint64_t asz = 0, aused = 0;
  if (free_b && arena_configured() && gpushare_shim_arena_stats(&asz, &aused)) {
    // with a broker arena: what its rest serves (every entry point allocates from it), plus what
    // the quota still lets the driver give
    uint64_t room = asz - aused;
    pthread_mutex_lock(&g_arena.mu);
    for (int i = 0; i < g_nwin; ++i)
      for (int sl = 0; sl < g_win[i].nslots; ++sl)
        if (g_win[i].slot_g[sl] >= 0) room += kWinAlign - g_win[i].slot_used[sl];
    pthread_mutex_unlock(&g_arena.mu);
    *free_b = (size_t)(room + *free_b);
    if (*free_b > quota) *free_b = (size_t)quota;
  }
  return e;
}

namespace {
uint64_t report_total(uint64_t real_total) {
  if (!enabled()) return real_total;
  if (!g.quota.load()) set_quota_from_device_bytes(real_total);
  uint64_t q = g.quota.load();
  return (q && real_total > q) ? q : real_total;
}
}  // namespace

GS_EXPORT hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t dev) {
  auto f = real_hipDeviceTotalMem();
  if (!f) return hipErrorNotInitialized;
  hipError_t e = f(bytes, dev);
  if (e == hipSuccess && bytes) *bytes = (size_t)report_total(*bytes);
  return e;
}

GS_EXPORT hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int dev) {
  auto f = real_hipGetDevicePropertiesR0600();
  if (!f) return hipErrorNotInitialized;
  hipError_t e = f(prop, dev);
  if (e == hipSuccess && prop) prop->totalGlobalMem = (size_t)report_total(prop->totalGlobalMem);
  return e;
}

GS_EXPORT hipError_t hipGetDevicePropertiesR0000(hipDeviceProp_tR0000* prop, int dev) {
  auto f = real_hipGetDevicePropertiesR0000();
  if (!f) return hipErrorNotInitialized;
  hipError_t e = f(prop, dev);
  if (e == hipSuccess && prop) prop->totalGlobalMem = (size_t)report_total(prop->totalGlobalMem);
  return e;
}

GS_EXPORT hipError_t hipGetDeviceProperties(hipDeviceProp_tR0000* prop, int dev) {
  auto f = real_hipGetDeviceProperties();
  if (!f) return hipErrorNotInitialized;
  hipError_t e = f(prop, dev);
  if (e == hipSuccess && prop) prop->totalGlobalMem = (size_t)report_total(prop->totalGlobalMem);
  return e;
}

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
