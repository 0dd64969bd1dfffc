// The libc ioctl and close interposers of the quota shim (kfd mode, the default): charges at the
// KFD boundary and on the amdgpu render node, and notes the KFD imports and queues this process
// makes (shim.h lists the units and the lock order).
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
// A GEM buffer still CPU-mapped after its GEM_CLOSE (the mapping holds it), and a DRM file held
// only by a process the shim cannot read in /proc, are not followed.
#include "shim.h"

#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

namespace gs {
namespace {

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
constexpr uint32_t kKfdVram = 1u << 0;  // KFD_IOC_ALLOC_MEM_FLAGS_VRAM
constexpr unsigned long kIocAlloc = kfd_ioc(3, 0x16, sizeof(KfdAllocArgs));  // AMDKFD_IOWR(0x16)
static_assert(sizeof(KfdAllocArgs) == 40 && sizeof(KfdFreeArgs) == 8, "KFD uapi layout");
struct KfdImportArgs {  // struct kfd_ioctl_import_dmabuf_args
  uint64_t va_addr;
  uint64_t handle;
  uint32_t gpu_id;
  uint32_t dmabuf_fd;
};
constexpr unsigned long kIocImport = kfd_ioc(3, 0x1D, sizeof(KfdImportArgs));  // AMDKFD_IOWR(0x1D)
static_assert(sizeof(KfdUnmapArgs) == 24 && sizeof(KfdImportArgs) == 24, "KFD uapi layout");
// AMDKFD_IOC_CREATE_QUEUE (0x02) / DESTROY_QUEUE (0x03). The create args grew over kernel
// versions (88 bytes, 96 with sdma_engine_id), so the request is matched by its type and number;
// queue_id is at offset 52 in every version.
constexpr unsigned long kIocNrMask = (0xffUL << 8) | 0xffUL;
constexpr unsigned long kIocCreateQueueNr = ((unsigned long)'K' << 8) | 0x02;
constexpr unsigned long kIocDestroyQueueNr = ((unsigned long)'K' << 8) | 0x03;
struct KfdDestroyQueueArgs {
  uint32_t queue_id, pad;
};
constexpr unsigned long kIocDestroyQueue = kfd_ioc(3, 0x03, sizeof(KfdDestroyQueueArgs));
constexpr size_t kQueueIdOffset = 52;

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

std::atomic<uint64_t> g_drm_client[kMaxDrmFd];  // fd -> its DRM client key + 1 (0: no charged GEM handles)
std::atomic<int> g_gem_live{0};                  // charged GEM handles in this process (fast path skip)
struct Lingering {                               // clients whose charged fd closed while still referred to
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  uint64_t client[64];
  int n = 0;
};
Lingering g_linger;

// ---- KFD boundary --------------------------------------------------------------------------
bool free_allocs_at_exit();
void alloc_note(int kfd, uint64_t handle, uint32_t gpu_id);

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
  if (free_allocs_at_exit()) alloc_note(fd, a->handle, a->gpu_id);
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

bool linger_has(uint64_t key) {
  pthread_mutex_lock(&g_linger.mu);
  bool have = false;
  for (int i = 0; i < g_linger.n; ++i) have |= g_linger.client[i] == key;
  pthread_mutex_unlock(&g_linger.mu);
  return have;
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

// ---- the runtime's KFD imports, and this process's queues ----
// HIP 7.0 (the runtime PyTorch bundles) never frees the KFD object it creates when it imports a
// dma-buf: after hipMemRelease the granule stays referenced until the process is torn down, and
// the broker cannot lend it to the next pod before that (tools/diag/dmabuf_ref_probe.cpp,
// profiles/r5/dmabuf_refs/). HIP 7.2 frees it at hipMemRelease. So the shim notes the imports the
// runtime makes while an import of the shim's is under way (a tag: the arena, or an IPC mapping),
// and at release frees the ones a runtime older than 7.1 left behind. At the fast exit (arena.cpp)
// it frees all of them, after destroying this process's queues.
struct KfdImport {
  uint64_t handle;
  int kfd;
  uint32_t gpu_id;
  int tag;  // 0: free slot
};
constexpr int kMaxImports = 4096;
KfdImport g_imports[kMaxImports];
std::atomic<int> g_nimports{0};  // slots in use (high-water mark)
std::atomic<int> g_imports_live{0};
pthread_mutex_t g_imp_mu = PTHREAD_MUTEX_INITIALIZER;

struct KfdQueue {
  std::atomic<int> kfd;    // -1: free slot
  std::atomic<uint32_t> id;
};
constexpr int kMaxQueues = 256;
KfdQueue g_queues[kMaxQueues];
std::atomic<int> g_nqueues{0};
std::atomic<bool> g_queue_init{false};

void queues_init() {
  if (g_queue_init.exchange(true)) return;
  for (auto& q : g_queues) q.kfd.store(-1);
}

// whether `fd` is /dev/kfd (a queue is created rarely: one readlink each)
bool is_kfd(int fd) {
  char path[64], link[32];
  snprintf(path, sizeof path, "/proc/self/fd/%d", fd);
  ssize_t n = readlink(path, link, sizeof link - 1);
  if (n <= 0) return false;
  link[n] = 0;
  return !strcmp(link, "/dev/kfd");
}

void queue_note(int kfd, uint32_t id) {
  queues_init();
  for (int i = 0; i < kMaxQueues; ++i) {
    int expect = -1;
    if (g_queues[i].kfd.load(std::memory_order_relaxed) == -1 && g_queues[i].kfd.compare_exchange_strong(expect, -2)) {
      g_queues[i].id.store(id);
      g_queues[i].kfd.store(kfd);
      int n = g_nqueues.load();
      while (i + 1 > n && !g_nqueues.compare_exchange_weak(n, i + 1)) {
      }
      return;
    }
  }
}

void queue_forget(int kfd, uint32_t id) {
  int n = g_nqueues.load();
  for (int i = 0; i < n; ++i)
    if (g_queues[i].kfd.load() == kfd && g_queues[i].id.load() == id) {
      g_queues[i].kfd.store(-1);
      return;
    }
}

void import_note(int kfd, const KfdImportArgs* a, int tag) {
  pthread_mutex_lock(&g_imp_mu);
  int n = g_nimports.load(std::memory_order_relaxed);
  int slot = -1;
  for (int i = 0; i < n && slot < 0; ++i)
    if (!g_imports[i].tag) slot = i;
  if (slot < 0 && n < kMaxImports) slot = n;
  if (slot >= 0) {
    g_imports[slot] = {a->handle, kfd, a->gpu_id, tag};
    if (slot == n) g_nimports.store(n + 1, std::memory_order_release);
    g_imports_live.fetch_add(1, std::memory_order_relaxed);
  }
  pthread_mutex_unlock(&g_imp_mu);
}

// every KFD allocation too (tag kTagAlloc), when GPUSHARE_SHIM_FREE_ALLOCS_AT_EXIT=1: the fast exit
// then frees the process's own buffers as well, before the kernel's release of the process
constexpr int kTagAlloc = 3;
bool free_allocs_at_exit() {
  static int v = -1;
  if (v < 0) v = env_u64("GPUSHARE_SHIM_FREE_ALLOCS_AT_EXIT", 0) ? 1 : 0;
  return v == 1;
}

void alloc_note(int kfd, uint64_t handle, uint32_t gpu_id) {
  KfdImportArgs a{};
  a.handle = handle;
  a.gpu_id = gpu_id;
  import_note(kfd, &a, kTagAlloc);
}

void import_forget(uint64_t handle) {
  pthread_mutex_lock(&g_imp_mu);
  int n = g_nimports.load(std::memory_order_relaxed);
  for (int i = 0; i < n; ++i)
    if (g_imports[i].tag && g_imports[i].handle == handle) {
      g_imports[i].tag = 0;
      g_imports_live.fetch_sub(1, std::memory_order_relaxed);
    }
  pthread_mutex_unlock(&g_imp_mu);
}

int free_import(ioctl_t f, KfdImport& m) {
  uint32_t dev = m.gpu_id;
  KfdUnmapArgs u{m.handle, reinterpret_cast<uint64_t>(&dev), 1, 0};
  (void)f(m.kfd, kIocUnmap, &u);  // mapped through VMM, not KFD: normally refused, harmless
  KfdFreeArgs fr{m.handle};
  return f(m.kfd, kIocFree, &fr) == 0;
}

int ioctl_body(ioctl_t f, int fd, unsigned long req, void* arg);

void kfd_atfork_child() {
  for (auto& fl : g_drm_client) fl.store(0, std::memory_order_relaxed);   // the parent's GEM handles are the parent's
  g_gem_live.store(0);
  pthread_mutex_init(&g_linger.mu, nullptr);
  g_linger.n = 0;
  pthread_mutex_init(&g_imp_mu, nullptr);   // the parent's imports and queues are the parent's
  g_nimports.store(0);
  g_imports_live.store(0);
  for (auto& q : g_queues) q.kfd.store(-1);
  g_nqueues.store(0);
}

__attribute__((constructor)) void kfd_register_atfork() {
  queues_init();
  pthread_atfork(nullptr, nullptr, kfd_atfork_child);
}
}  // namespace

thread_local int t_import_tag = 0;

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

// free the imports of `tag` the runtime kept (after it released the handles); returns how many
int imports_free(int tag) {
  ioctl_t f = real_ioctl();
  if (!f) return 0;
  int n = 0;
  pthread_mutex_lock(&g_imp_mu);
  int top = g_nimports.load(std::memory_order_relaxed);
  for (int i = 0; i < top; ++i) {
    KfdImport& m = g_imports[i];
    if (m.tag != tag) continue;
    n += free_import(f, m);
    m.tag = 0;
    g_imports_live.fetch_sub(1, std::memory_order_relaxed);
  }
  pthread_mutex_unlock(&g_imp_mu);
  return n;
}

int imports_live() { return g_imports_live.load(std::memory_order_relaxed); }

// The fast exit (arena.cpp): every queue of this process goes, the way the kernel destroys them
// when the process exits, so nothing on the GPU can touch this process's memory any more.
int queues_destroy_all() {
  ioctl_t f = real_ioctl();
  if (!f) return 0;
  int n = 0, top = g_nqueues.load();
  for (int i = 0; i < top; ++i) {
    int kfd = g_queues[i].kfd.load();
    if (kfd < 0) continue;
    KfdDestroyQueueArgs d{g_queues[i].id.load(), 0};
    n += f(kfd, kIocDestroyQueue, &d) == 0;
    g_queues[i].kfd.store(-1);
  }
  return n;
}

// ... then every import noted (the queues are gone: nothing uses them), without waiting for a
// lock a thread of the dying process may hold for ever: a trylock for up to 200 ms, then without
int imports_free_all_unlocked() {
  ioctl_t f = real_ioctl();
  if (!f) return 0;
  bool locked = false;
  for (int k = 0; k < 200 && !(locked = pthread_mutex_trylock(&g_imp_mu) == 0); ++k) usleep(1000);
  int n = 0, top = g_nimports.load(std::memory_order_acquire);
  for (int i = 0; i < top; ++i) {
    KfdImport& m = g_imports[i];
    if (!m.tag) continue;
    n += free_import(f, m);
    m.tag = 0;
  }
  g_imports_live.store(0);
  if (locked) pthread_mutex_unlock(&g_imp_mu);
  return n;
}

}  // namespace gs

using namespace gs;

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
  if (req == kIocImport && arg && t_import_tag) {
    int r = f(fd, req, arg);
    if (r == 0) import_note(fd, static_cast<KfdImportArgs*>(arg), t_import_tag);
    return r;
  }
  if ((req & kIocNrMask) == kIocCreateQueueNr && (req >> 30) == 3 && ((req >> 16) & 0x3fff) >= 88 && arg) {
    int r = f(fd, req, arg);
    if (r == 0 && is_kfd(fd)) {
      uint32_t id;
      memcpy(&id, static_cast<char*>(arg) + kQueueIdOffset, sizeof id);
      queue_note(fd, id);
    }
    return r;
  }
  if ((req & kIocNrMask) == kIocDestroyQueueNr && arg) {
    uint32_t id = static_cast<KfdDestroyQueueArgs*>(arg)->queue_id;
    int r = f(fd, req, arg);
    if (r == 0) queue_forget(fd, id);
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

namespace gs {
namespace {
int ioctl_body(ioctl_t f, int fd, unsigned long req, void* arg) {
  // Cheap filters first, and never the once-control while init() runs (the runtime may start
  // up underneath it and allocate through here: waiting on that init would deadlock).
  if ((req != kIocAlloc && req != kIocFree && req != kDrmGemCreate && req != kDrmGemClose &&
       req != kDrmPrimeHandleToFd) || !arg || env_mode() != kModeKfd || g_initializing.load(std::memory_order_acquire))
    return f(fd, req, arg);
  if (req == kIocAlloc && !(static_cast<KfdAllocArgs*>(arg)->flags & kKfdVram)) {
    int r = f(fd, req, arg);
    if (r == 0 && free_allocs_at_exit()) {
      auto* a = static_cast<KfdAllocArgs*>(arg);
      alloc_note(fd, a->handle, a->gpu_id);
    }
    return r;
  }
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
}  // namespace gs

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
