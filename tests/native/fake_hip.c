// Stub HIP runtime for CPU-only tests of the quota shim (same soname as ROCm's runtime).
// Like the real one it gets device memory from the KFD: every allocation below is an
// AMDKFD_IOC_ALLOC_MEMORY_OF_GPU ioctl (VRAM flag) issued through libc's ioctl — which the
// preloaded shim intercepts — and this library also exports the ioctl that emulates /dev/kfd
// (the shim forwards to it via RTLD_NEXT), with a 16 GiB "device". Pools (hipMallocAsync)
// keep freed blocks until trimmed, and fake_runtime_scratch() allocates behind the API's back
// the way ROCr allocates scratch: the shapes of HBM use the HIP entry points cannot see.
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <stdio.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <time.h>
typedef int hipError_t;
struct kfd_alloc { uint64_t va, size, handle, mmap_offset; uint32_t gpu_id, flags; };
struct kfd_free { uint64_t handle; };
#define KIOC(dir, nr, sz) (((unsigned long)(dir) << 30) | ((unsigned long)(sz) << 16) | ((unsigned long)'K' << 8) | (nr))
#define KFD_ALLOC KIOC(3, 0x16, sizeof(struct kfd_alloc))
#define KFD_FREE KIOC(1, 0x17, sizeof(struct kfd_free))
/* AMDKFD_IOC_IMPORT_DMABUF: the "kernel" keeps the dma-buf referenced (a dup of the fd) until the
   import is freed (AMDKFD_IOC_FREE_MEMORY_OF_GPU of its handle) */
struct kfd_import { uint64_t va, handle; uint32_t gpu_id, dmabuf_fd; };
#define KFD_IMPORT KIOC(3, 0x1D, sizeof(struct kfd_import))
#define IMPORT_HANDLE (1ull << 40)
#define MAXIMP 4096
static int g_imp_fd[MAXIMP];  /* fd + 1 of each live import, 0 none */
static unsigned g_imp_next = 0;
#define MAXH (1 << 20)
static size_t g_total = (size_t)16 << 30, g_used = 0;
static uint64_t g_sizes[MAXH];
static uint64_t g_next = 1;

/* amdgpu render node: DRM_IOCTL_AMDGPU_GEM_CREATE / DRM_IOCTL_GEM_CLOSE */
struct gem_create { uint64_t bo_size, alignment, domains, domain_flags; };
struct gem_close { uint32_t handle, pad; };
#define DIOC(dir, nr, sz) (((unsigned long)(dir) << 30) | ((unsigned long)(sz) << 16) | ((unsigned long)'d' << 8) | (nr))
#define GEM_CREATE DIOC(3, 0x40, sizeof(struct gem_create))
#define GEM_CLOSE DIOC(1, 0x09, sizeof(struct gem_close))
static uint64_t g_gem_sizes[4096];
static uint32_t g_gem_next = 1;

/* The kernel's view of a closed fd: with a synthetic /proc (GPUSHARE_SHIM_PROC_ROOT, the shim
   tests) its fd and fdinfo entries disappear when the fd really closes. */
int close(int fd) {
  const char* root = getenv("GPUSHARE_SHIM_PROC_ROOT");
  if (root && fd >= 0) {
    char p[512];
    snprintf(p, sizeof p, "%s/%d/fd/%d", root, (int)getpid(), fd); unlink(p);
    snprintf(p, sizeof p, "%s/%d/fdinfo/%d", root, (int)getpid(), fd); unlink(p);
  }
  return (int)syscall(SYS_close, fd);
}

int ioctl(int fd, unsigned long req, ...) {
  va_list ap; va_start(ap, req); void* arg = va_arg(ap, void*); va_end(ap);
  if (req == GEM_CREATE) {
    struct gem_create* a = (struct gem_create*)arg;
    uint64_t n = a->bo_size, vram = a->domains & 0x4;
    if (vram && __atomic_add_fetch(&g_used, n, __ATOMIC_ACQ_REL) > g_total) {
      __atomic_fetch_sub(&g_used, n, __ATOMIC_ACQ_REL); errno = ENOMEM; return -1;
    }
    uint32_t h = __atomic_fetch_add(&g_gem_next, 1, __ATOMIC_ACQ_REL) % 4096;
    g_gem_sizes[h] = vram ? n : 0;
    memset(a, 0, sizeof *a); *(uint32_t*)a = h; return 0;
  }
  if (req == DIOC(3, 0x2d, 12)) {           /* DRM_IOCTL_PRIME_HANDLE_TO_FD: a dma-buf fd */
    ((int32_t*)arg)[2] = dup(fd); return 0;
  }
  if (req == GEM_CLOSE) {
    uint32_t h = ((struct gem_close*)arg)->handle % 4096;
    __atomic_fetch_sub(&g_used, __atomic_exchange_n(&g_gem_sizes[h], 0, __ATOMIC_ACQ_REL), __ATOMIC_ACQ_REL);
    return 0;
  }
  if (req == KFD_ALLOC) {
    struct kfd_alloc* a = (struct kfd_alloc*)arg;
    size_t cur = __atomic_load_n(&g_used, __ATOMIC_RELAXED);
    do { if (cur + a->size > g_total) { errno = ENOMEM; return -1; } }
    while (!__atomic_compare_exchange_n(&g_used, &cur, cur + a->size, 1, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED));
    uint64_t h = __atomic_fetch_add(&g_next, 1, __ATOMIC_ACQ_REL) % MAXH;
    __atomic_store_n(&g_sizes[h], a->size, __ATOMIC_RELEASE);
    a->handle = h; return 0;
  }
  if (req == KFD_IMPORT) {
    struct kfd_import* a = (struct kfd_import*)arg;
    unsigned i = __atomic_fetch_add(&g_imp_next, 1, __ATOMIC_ACQ_REL) % MAXIMP;
    g_imp_fd[i] = (int)a->dmabuf_fd + 1;
    a->handle = IMPORT_HANDLE | i; return 0;
  }
  if (req == KFD_FREE && (((struct kfd_free*)arg)->handle & IMPORT_HANDLE)) {
    unsigned i = (unsigned)(((struct kfd_free*)arg)->handle & (MAXIMP - 1));
    if (g_imp_fd[i] <= 0) { errno = EINVAL; return -1; }
    close(g_imp_fd[i] - 1); g_imp_fd[i] = 0; return 0;
  }
  if (req == KFD_FREE) {
    uint64_t h = ((struct kfd_free*)arg)->handle;
    __atomic_fetch_sub(&g_used, __atomic_exchange_n(&g_sizes[h], 0, __ATOMIC_ACQ_REL), __ATOMIC_ACQ_REL);
    return 0;
  }
  int (*real)(int, unsigned long, ...) = (int (*)(int, unsigned long, ...))dlsym(RTLD_NEXT, "ioctl");
  return real(fd, req, arg);
}
/* FAKE_HIP_PROBE_FIXED=1: the runtime's address-space habit measured on MI355X — it finds a
   free range (map + unmap), issues the allocation ioctl, then maps that range MAP_FIXED and
   trims it. Whatever the process mapped inside the range meanwhile (the shim initialising
   inside that ioctl) is silently replaced. */
/* FAKE_HIP_HELD_GIB / FAKE_HIP_HELD_MS: that much of the device is held by "another process"
   (pods of a previous broker) until that many ms after start */
static size_t g_held = 0;
static double g_held_until = 0;
/* FAKE_HIP_LATE_GIB / FAKE_HIP_LATE_MS / FAKE_HIP_LATE_FOR_MS: "another process" takes that much
   of the device that many ms after start, and gives it back after FOR_MS (0: keeps it) — driver
   pressure on a broker that holds the rest */
static size_t g_late = 0;
static double g_late_at = 0, g_late_until = 0;
static int g_late_state = 0;
static double fake_now(void);
static void total_init(void) {     /* FAKE_HIP_TOTAL_GIB: the "device" size (default 16 GiB) */
  static int done = 0;
  if (__atomic_exchange_n(&done, 1, __ATOMIC_ACQ_REL)) return;
  const char* tg = getenv("FAKE_HIP_TOTAL_GIB");
  if (tg && atof(tg) > 0) g_total = (size_t)(atof(tg) * (double)(1ull << 30));
  const char* hg = getenv("FAKE_HIP_HELD_GIB");
  const char* hm = getenv("FAKE_HIP_HELD_MS");
  if (hg && atof(hg) > 0) {
    g_held = (size_t)(atof(hg) * (double)(1ull << 30));
    __atomic_add_fetch(&g_used, g_held, __ATOMIC_ACQ_REL);
    g_held_until = fake_now() + (hm ? atof(hm) : 0) / 1e3;
  }
  const char* lg = getenv("FAKE_HIP_LATE_GIB");
  if (lg && atof(lg) > 0) {
    const char* lm = getenv("FAKE_HIP_LATE_MS");
    const char* lf = getenv("FAKE_HIP_LATE_FOR_MS");
    g_late = (size_t)(atof(lg) * (double)(1ull << 30));
    g_late_at = fake_now() + (lm ? atof(lm) : 0) / 1e3;
    g_late_until = lf && atof(lf) > 0 ? g_late_at + atof(lf) / 1e3 : 0;
  }
}
static void late_tick(void) {
  double t = fake_now();
  if (g_late_state == 0 && g_late && t >= g_late_at) { __atomic_add_fetch(&g_used, g_late, __ATOMIC_ACQ_REL); g_late_state = 1; }
  if (g_late_state == 1 && g_late_until > 0 && t >= g_late_until) { __atomic_fetch_sub(&g_used, g_late, __ATOMIC_ACQ_REL); g_late_state = 2; }
}
static void held_release(void) {
  if (g_held && fake_now() >= g_held_until) { __atomic_fetch_sub(&g_used, g_held, __ATOMIC_ACQ_REL); g_held = 0; }
}
static int kfd(size_t n, uint64_t* h) {
  total_init();
  late_tick();
  struct kfd_alloc a = {0, n, 0, 0, 1, 1u /* VRAM */};
  const char* pf = getenv("FAKE_HIP_PROBE_FIXED");
  void* probe = NULL;
  if (pf && *pf == '1') {
    probe = mmap(NULL, 2 * 4096, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (probe == MAP_FAILED) probe = NULL; else munmap(probe, 2 * 4096);
  }
  int r = ioctl(3, KFD_ALLOC, &a);
  if (probe) {
    mmap(probe, 2 * 4096, PROT_READ, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED, -1, 0);
    munmap((char*)probe + 4096, 4096);
  }
  if (r) return 2;                                   /* hipErrorOutOfMemory */
  *h = a.handle; return 0;
}
static void kfd_release(uint64_t h) { struct kfd_free f = {h}; ioctl(3, KFD_FREE, &f); }
#define PTR(h) ((void*)(uintptr_t)((h) << 12))
#define HANDLE(p) ((uint64_t)(uintptr_t)(p) >> 12)
hipError_t hipMalloc(void** p, size_t n) { uint64_t h; int e = kfd(n, &h); if (!e) *p = PTR(h); return e; }
hipError_t hipExtMallocWithFlags(void** p, size_t n, unsigned f) { return hipMalloc(p, n); }
hipError_t hipMallocManaged(void** p, size_t n, unsigned f) { return hipMalloc(p, n); }
hipError_t hipFree(void* p) { if (p) kfd_release(HANDLE(p)); return 0; }
/* stream-ordered pool: freed blocks stay cached (and charged) until hipMemPoolTrimTo */
static struct { uint64_t h, n; } g_pool[4096];
static int g_npool = 0;
hipError_t hipMallocAsync(void** p, size_t n, void* s) {
  for (int i = 0; i < g_npool; ++i) if (g_pool[i].n >= n) { *p = PTR(g_pool[i].h); g_pool[i] = g_pool[--g_npool]; return 0; }
  return hipMalloc(p, n);
}
hipError_t hipFreeAsync(void* p, void* s) {
  if (!p) return 0;
  if (g_npool < 4096) { g_pool[g_npool].h = HANDLE(p); g_pool[g_npool].n = g_sizes[HANDLE(p)]; g_npool++; return 0; }
  return hipFree(p);
}
hipError_t hipMemPoolTrimTo(void* pool, size_t keep) {
  size_t cached = 0; for (int i = 0; i < g_npool; ++i) cached += g_pool[i].n;
  while (g_npool && cached > keep) { --g_npool; cached -= g_pool[g_npool].n; kfd_release(g_pool[g_npool].h); }
  return 0;
}
/* FAKE_HIP_INIT_KFD=1: the first call initialises the "runtime", which allocates VRAM through
   the KFD ioctl the way ROCr does while the shim may still be inside its own init */
static int g_inited = 0;
static void runtime_init(void) {
  if (__atomic_exchange_n(&g_inited, 1, __ATOMIC_ACQ_REL)) return;
  const char* v = getenv("FAKE_HIP_INIT_KFD");
  if (v && *v == '1') { uint64_t h; kfd((size_t)2 << 20, &h); }
}
hipError_t hipMemGetInfo(size_t* f, size_t* t) {
  total_init(); held_release(); late_tick(); runtime_init();
  size_t u = __atomic_load_n(&g_used, __ATOMIC_ACQUIRE);
  *f = u < g_total ? g_total - u : 0; *t = g_total; return 0;
}
hipError_t hipDeviceTotalMem(size_t* b, int d) { total_init(); *b = g_total; return 0; }
hipError_t hipMemCreate(uint64_t* h, size_t n, const void* prop, unsigned long long fl) { return kfd(n, h); }
hipError_t hipMemRelease_imported(uint64_t h);
hipError_t hipMemRelease(uint64_t h) { if (h & (1ull << 62)) return hipMemRelease_imported(h); kfd_release(h); return 0; }
/* what ROCr does for a scratch-heavy dispatch: VRAM taken inside the runtime, no HIP call */
int fake_runtime_scratch(size_t n) { uint64_t h; return kfd(n, &h); }
/* HIP VMM for the shim's HBM-broker arena: an import goes through the KFD import ioctl with a dup
   of the broker's fd (the "kernel" reference; the high bit marks the handle); the address range is
   a host reservation. Import follows the 7.2 runtime: the fd is the pointer's value, and an
   address (a pointer to the fd) is refused with hipErrorInvalidValue. Release frees the KFD
   import from 7.1 on; below 7.1 it leaves it, as HIP 7.0 does (measured on MI355X,
   profiles/r5/dmabuf_refs/), so the reference stays until the process exits. */
#define IMPORTED (1ull << 62)
/* FAKE_HIP_VERSION (default 70253211, a 7.2 runtime): below 7.1 the import reads the fd through
   the pointer as HIP 7.0 does (and "crashes" — exit 139 — on a bare value); from 7.1 on it takes
   the pointer's value and refuses an address */
static int fake_version(void) { const char* v = getenv("FAKE_HIP_VERSION"); return v ? atoi(v) : 70253211; }
hipError_t hipRuntimeGetVersion(int* v) { *v = fake_version(); return 0; }
hipError_t hipMemImportFromShareableHandle(uint64_t* h, void* os, int type) {
  uintptr_t fd = (uintptr_t)os;
  if (fake_version() < 70100000) {
    if (fd < (1u << 20)) _exit(139);                 /* HIP 7.0 dereferences a bare fd value */
    fd = (uintptr_t)*(int*)os;
  } else if (fd > (1u << 20)) {
    return 1;                                        /* hipErrorInvalidValue */
  }
  int d = dup((int)fd);
  if (d < 0) return 1;
  struct kfd_import a = {0, 0, 1, (uint32_t)d};
  if (ioctl(3, KFD_IMPORT, &a)) { close(d); return 1; }
  *h = IMPORTED | a.handle; return 0;
}
int fake_live_imports(void) { int n = 0; for (int i = 0; i < MAXIMP; ++i) n += g_imp_fd[i] > 0; return n; }
hipError_t hipMemRelease_imported(uint64_t h) {
  if (fake_version() >= 70100000) { struct kfd_free f = {h & ~IMPORTED}; ioctl(3, KFD_FREE, &f); }
  return 0;
}
/* FAKE_HIP_RESERVE_ALIGN_MAX=<bytes>: like HIP 7.x, a larger alignment is not honoured, and the
   range is deliberately placed off any larger boundary */
hipError_t hipMemAddressReserve(void** p, size_t n, size_t al, void* addr, unsigned long long fl) {
  if (al < 4096) al = 4096;
  const char* cap = getenv("FAKE_HIP_RESERVE_ALIGN_MAX");
  size_t skew = 0;
  if (cap && al > strtoull(cap, 0, 10)) { al = strtoull(cap, 0, 10); skew = al; }
  char* m = mmap(0, n + al + skew, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (m == MAP_FAILED) return 2;
  char* a = (char*)(((uintptr_t)m + al - 1) / al * al);      /* honour the alignment: trim both ends */
  if (skew && ((uintptr_t)a % (1ull << 30)) == 0) a += skew;
  if (a > m) munmap(m, (size_t)(a - m));
  if (m + n + al + skew > a + n) munmap(a + n, (size_t)(m + n + al + skew - (a + n)));
  *p = a; return 0;
}
hipError_t hipMemAddressFree(void* p, size_t n) { munmap(p, n); return 0; }
hipError_t hipMemMap(void* p, size_t n, size_t off, uint64_t h, unsigned long long fl) { return 0; }
hipError_t hipMemUnmap(void* p, size_t n) { return 0; }
/* FAKE_HIP_ACCESS_REFUSE_SIZE=<bytes>: refuse an access call of exactly that size, as HIP 7.x
   now and then refuses one driver page's access (hipErrorInvalidValue) */
hipError_t hipMemSetAccess(void* p, size_t n, const void* d, size_t c) {
  const char* r = getenv("FAKE_HIP_ACCESS_REFUSE_SIZE");
  return r && strtoull(r, 0, 10) == n ? 1 : 0;
}
hipError_t hipGetDevice(int* d) { *d = 0; return 0; }
hipError_t hipDeviceSynchronize(void) { return 0; }
/* what the HBM broker (native/hbmbroker) needs besides the above: exported handles are memfds,
   the scrub (hipMemsetAsync) is counted, not performed (the reserved range is not accessible) */
hipError_t hipMemGetAllocationGranularity(size_t* g, const void* prop, int opt) { *g = 4096; return 0; }
hipError_t hipMemExportToShareableHandle(void* out, uint64_t h, int type, unsigned long long fl) {
  int fd = (int)syscall(SYS_memfd_create, "fake-vram", 0);
  if (fd < 0) return 1;
  *(int*)out = fd; return 0;
}
static size_t g_memset_bytes = 0;
/* FAKE_HIP_MEMSET_MS_PER_GIB: the stream zeroes at that pace, one memset after another; an event
   recorded after them completes when they have */
static double g_stream_busy = 0;
static double fake_now(void);
hipError_t hipMemsetAsync(void* p, int v, size_t n, void* s) {
  __atomic_add_fetch(&g_memset_bytes, n, __ATOMIC_RELAXED);
  const char* pace = getenv("FAKE_HIP_MEMSET_MS_PER_GIB");
  if (pace) {
    double t = fake_now(), start = g_stream_busy > t ? g_stream_busy : t;
    g_stream_busy = start + (double)n / (double)(1ull << 30) * atof(pace) / 1e3;
  }
  return 0;
}
hipError_t hipStreamCreateWithFlags(void** s, unsigned f) { *s = (void*)0x1; return 0; }
/* no code objects here: the broker zeroes with hipMemsetAsync */
hipError_t hipModuleLoad(void** m, const char* path) { return 1; }
hipError_t hipModuleGetFunction(void** f, void* m, const char* name) { return 1; }
hipError_t hipModuleLaunchKernel(void* f, unsigned gx, unsigned gy, unsigned gz, unsigned bx, unsigned by, unsigned bz,
                                 unsigned shm, void* s, void** params, void** extra) { return 1; }
hipError_t hipGetLastError(void) { return 0; }
hipError_t hipStreamSynchronize(void* s) {
  double w = g_stream_busy - fake_now();
  if (w > 0) { struct timespec t = {(time_t)w, (long)((w - (time_t)w) * 1e9)}; nanosleep(&t, 0); }
  return 0;
}
hipError_t hipSetDevice(int d) { return 0; }
hipError_t hipDeviceGetByPCIBusId(int* d, const char* bdf) { *d = 0; return 0; }
const char* hipGetErrorString(hipError_t e) { return "fake hip error"; }
/* events: hipEventRecord completes FAKE_HIP_EVENT_MS after it was recorded (0 = at once), so a
   test can hold the broker's asynchronous scrub, or a stream-ordered free, in flight */
struct fake_event { double done_at; };
static double fake_now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }  /* (declared above) */
hipError_t hipEventCreateWithFlags(void** e, unsigned f) {
  struct fake_event* ev = calloc(1, sizeof *ev);
  if (!ev) return 2;
  *e = ev; return 0;
}
hipError_t hipEventCreate(void** e) { return hipEventCreateWithFlags(e, 0); }
hipError_t hipEventRecord(void* e, void* s) {
  const char* ms = getenv("FAKE_HIP_EVENT_MS");
  double at = fake_now() + (ms ? atof(ms) : 0.0) / 1e3;
  ((struct fake_event*)e)->done_at = g_stream_busy > at ? g_stream_busy : at;
  return 0;
}
hipError_t hipEventQuery(void* e) { return fake_now() >= ((struct fake_event*)e)->done_at ? 0 : 600; /* hipErrorNotReady */ }
hipError_t hipEventSynchronize(void* e) {
  double w = ((struct fake_event*)e)->done_at - fake_now();
  if (w > 0) { struct timespec t = {(time_t)w, (long)((w - (time_t)w) * 1e9)}; nanosleep(&t, 0); }
  return 0;
}
hipError_t hipEventDestroy(void* e) { free(e); return 0; }
/* stream capture never on; the default pool is a token (hipMallocFromPoolAsync = hipMallocAsync) */
hipError_t hipStreamIsCapturing(void* s, int* st) { *st = 0; return 0; }
hipError_t hipDeviceGetDefaultMemPool(void** pool, int dev) { *pool = (void*)0x1; return 0; }
hipError_t hipMallocFromPoolAsync(void** p, size_t n, void* pool, void* s) { return hipMallocAsync(p, n, s); }
hipError_t hipMemGetAllocationPropertiesFromHandle(void* prop, uint64_t h) { return 1; }
/* what the runtime answers for arena memory (VMM mappings of imported dma-bufs), measured on MI355X
   (profiles/r6/arena_probe.jsonl): hipIpcGetMemHandle refuses it; hipMemRetainAllocationHandle
   hands out the mapping's handle — the broker's granule, which the caller could release */
hipError_t hipIpcGetMemHandle(void* h, void* p) { return 1; }
hipError_t hipIpcOpenMemHandle(void** p, char h[64], unsigned f) { return 1; }
hipError_t hipIpcCloseMemHandle(void* p) { return 1; }
hipError_t hipMemGetAddressRange(void** b, size_t* n, void* p) { if (b) *b = (void*)((uintptr_t)p & ~((1ull << 30) - 1)); if (n) *n = 1ull << 30; return 0; }
hipError_t hipMemRetainAllocationHandle(uint64_t* h, void* p) { *h = IMPORTED | 1; return 0; }
hipError_t hipStreamCreate(void** s) { *s = calloc(1, 8); return 0; }
hipError_t hipStreamCreateWithPriority(void** s, unsigned f, int pr) { *s = calloc(1, 8); return 0; }
hipError_t hipStreamDestroy(void* s) { return 0; }
