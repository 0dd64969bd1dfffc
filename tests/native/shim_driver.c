// Test driver: executes allocation commands against the (stub or real) HIP runtime and
// prints one JSON line per command. Linked against libamdhip64.so.7 like any HIP program.
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/ioctl.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>
static int g_render_fd = -1, g_dup_fd = -1, g_hold_pipe = -1;
static pid_t g_hold_pid = -1;
static int g_hold_fd = -1;
static unsigned long long g_cid = 0;
/* synthetic /proc entries (GPUSHARE_SHIM_PROC_ROOT) for fd of pid: <root>/<pid>/fd/<fd> -> a
   render node, <root>/<pid>/fdinfo/<fd> with drm-client-id; cid 0 removes them */
static void fake_fd(pid_t pid, int fd, unsigned long long cid) {
  const char* root = getenv("GPUSHARE_SHIM_PROC_ROOT");
  if (!root || fd < 0) return;
  char p[512], q[512];
  snprintf(p, sizeof p, "%s/%d", root, (int)pid); mkdir(p, 0755);
  snprintf(p, sizeof p, "%s/%d/fd", root, (int)pid); mkdir(p, 0755);
  snprintf(p, sizeof p, "%s/%d/fdinfo", root, (int)pid); mkdir(p, 0755);
  snprintf(p, sizeof p, "%s/%d/fd/%d", root, (int)pid, fd);
  snprintf(q, sizeof q, "%s/%d/fdinfo/%d", root, (int)pid, fd);
  unlink(p); unlink(q);
  if (!cid) return;
  if (symlink("/dev/dri/renderD128", p)) return;
  FILE* f = fopen(q, "w");
  if (f) { fprintf(f, "pos:\t0\nflags:\t02100002\ndrm-driver:\tamdgpu\ndrm-client-id:\t%llu\n", cid); fclose(f); }
}
static int fake_exists(pid_t pid, int fd) {
  const char* root = getenv("GPUSHARE_SHIM_PROC_ROOT");
  char q[512]; snprintf(q, sizeof q, "%s/%d/fdinfo/%d", root ? root : "/nonexistent", (int)pid, fd);
  return access(q, F_OK) == 0;
}
typedef int hipError_t;
hipError_t hipMalloc(void**, size_t); hipError_t hipFree(void*);
hipError_t hipMemGetInfo(size_t*, size_t*); hipError_t hipMallocAsync(void**, size_t, void*);
hipError_t hipFreeAsync(void*, void*); hipError_t hipMemCreate(uint64_t*, size_t, const void*, unsigned long long);
hipError_t hipMemRelease(uint64_t); hipError_t hipMemPoolTrimTo(void*, size_t); int fake_runtime_scratch(size_t);
hipError_t hipMemAddressReserve(void**, size_t, size_t, void*, unsigned long long); hipError_t hipMemAddressFree(void*, size_t);
hipError_t hipMemMap(void*, size_t, size_t, uint64_t, unsigned long long); hipError_t hipMemUnmap(void*, size_t);
hipError_t hipMemSetAccess(void*, size_t, const void*, size_t);
hipError_t hipMallocFromPoolAsync(void**, size_t, void*, void*); hipError_t hipDeviceGetDefaultMemPool(void**, int);
/* hipMemAllocationProp / hipMemAccessDesc as laid out in hip/hip_runtime_api.h, driver_types.h */
struct vprop { int type; int htype; struct { int type; int id; } loc; void* w32; unsigned char ct, rdma; unsigned short usage; };
struct vaccess { struct { int type; int id; } loc; int flags; };
/* VMM the way PyTorch's expandable segments use it: one reserved range, pages mapped one after another */
static char* g_vbase = 0; static size_t g_vsize = 0, g_vcur = 0;
static struct { char* va; uint64_t h; size_t n; } g_vpages[8192]; static int g_nv = 0;
// "threads N ITERS SIZE": N threads each alloc+free SIZE bytes ITERS times (quota contention)
struct targ { int iters; size_t n; int ok, denied; };
static void* worker(void* v) {
  struct targ* a = (struct targ*)v;
  for (int k = 0; k < a->iters; ++k) {
    void* p = 0;
    if (hipMalloc(&p, a->n) == 0) { a->ok++; hipFree(p); } else a->denied++;
  }
  return 0;
}
typedef int (*stats_fn)(uint64_t*, uint64_t*, uint64_t*, uint64_t*);
/* IPC (hip_runtime_api.h: hipIpcMemHandle_t is 64 bytes, passed by value to hipIpcOpenMemHandle) */
typedef struct { char reserved[64]; } ipch_t;
hipError_t hipIpcGetMemHandle(ipch_t*, void*); hipError_t hipIpcOpenMemHandle(void**, ipch_t, unsigned);
hipError_t hipIpcCloseMemHandle(void*); hipError_t hipMemGetAddressRange(void**, size_t*, void*);
hipError_t hipMemRetainAllocationHandle(uint64_t*, void*);
static double now_ms(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec * 1e3 + t.tv_nsec / 1e6; }
static void on_term(int sig) { (void)sig; const char m[] = "{\"op\":\"handled\"}\n"; ssize_t r = write(1, m, sizeof m - 1); (void)r; _exit(0); }
int main(int argc, char** argv) {
  void* ptrs[4096]; int np = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "alloc")) { size_t n = strtoull(argv[++i], 0, 10); void* p = 0; int e = hipMalloc(&p, n);
      printf("{\"op\":\"alloc\",\"n\":%zu,\"err\":%d,\"idx\":%d,\"p\":%llu}\n", n, e, e ? -1 : np,
             (unsigned long long)(uintptr_t)p); if (!e) ptrs[np++] = p; }
    else if (!strcmp(argv[i], "arena")) { int (*f)(uint64_t*, uint64_t*) = (int (*)(uint64_t*, uint64_t*))dlsym(RTLD_DEFAULT, "gpushare_shim_arena_stats");
      uint64_t sz = 0, used = 0; int on = f ? f(&sz, &used) : -2;
      printf("{\"op\":\"arena\",\"on\":%d,\"size\":%llu,\"used\":%llu}\n", on, (unsigned long long)sz, (unsigned long long)used); }
    else if (!strcmp(argv[i], "arenastream")) {
      typedef uint64_t* P;
      int (*f)(P, P, P, P, P, P, P, P, P) = (int (*)(P, P, P, P, P, P, P, P, P))dlsym(RTLD_DEFAULT, "gpushare_shim_arena_stream");
      uint64_t w = 0, wn = 0, m = 0, mn = 0, mp = 0, gr = 0, fi = 0, rn = 0, an = 0;
      int on = f ? f(&w, &wn, &m, &mn, &mp, &gr, &fi, &rn, &an) : -2;
      printf("{\"op\":\"arenastream\",\"on\":%d,\"waits\":%llu,\"wait_ms\":%.1f,\"msgs\":%llu,\"mapped\":%llu,\"granted\":%llu,\"first\":%llu}\n",
             on, (unsigned long long)w, wn / 1e6, (unsigned long long)m, (unsigned long long)mp, (unsigned long long)gr,
             (unsigned long long)fi); }
    else if (!strcmp(argv[i], "imports")) { int (*f)(void) = (int (*)(void))dlsym(RTLD_DEFAULT, "fake_live_imports");
      printf("{\"op\":\"imports\",\"live\":%d}\n", f ? f() : -2); }
    else if (!strcmp(argv[i], "arenarelease")) { int (*f)(void) = (int (*)(void))dlsym(RTLD_DEFAULT, "gpushare_shim_arena_release");
      printf("{\"op\":\"arenarelease\",\"r\":%d}\n", f ? f() : -2); fflush(stdout); }
    else if (!strcmp(argv[i], "sleepms")) { fflush(stdout); usleep((useconds_t)atoi(argv[++i]) * 1000); }
    else if (!strcmp(argv[i], "async")) { size_t n = strtoull(argv[++i], 0, 10); void* p = 0; int e = hipMallocAsync(&p, n, 0);
      printf("{\"op\":\"async\",\"n\":%zu,\"err\":%d,\"idx\":%d,\"p\":%llu}\n", n, e, e ? -1 : np,
             (unsigned long long)(uintptr_t)p); if (!e) ptrs[np++] = p; }
    else if (!strcmp(argv[i], "vmm")) { size_t n = strtoull(argv[++i], 0, 10); uint64_t h = 0; int e = hipMemCreate(&h, n, 0, 0);
      printf("{\"op\":\"vmm\",\"n\":%zu,\"err\":%d}\n", n, e); if (!e) hipMemRelease(h); }
    else if (!strcmp(argv[i], "freeasync")) { int k = atoi(argv[++i]); int e = hipFreeAsync(ptrs[k], 0); ptrs[k] = 0;
      printf("{\"op\":\"freeasync\",\"idx\":%d,\"err\":%d}\n", k, e); }
    else if (!strcmp(argv[i], "trim")) { int e = hipMemPoolTrimTo(0, 0); printf("{\"op\":\"trim\",\"err\":%d}\n", e); }
    else if (!strcmp(argv[i], "scratch")) { size_t n = strtoull(argv[++i], 0, 10); int e = fake_runtime_scratch(n);
      printf("{\"op\":\"scratch\",\"n\":%zu,\"err\":%d}\n", n, e); }
    else if (!strcmp(argv[i], "mode")) { int (*f)(void) = (int (*)(void))dlsym(RTLD_DEFAULT, "gpushare_shim_mode");
      printf("{\"op\":\"mode\",\"mode\":%d}\n", f ? f() : -2); }
    else if (!strcmp(argv[i], "fork")) { fflush(stdout); pid_t c = fork();
      if (c == 0) { size_t n = strtoull(argv[i + 1], 0, 10); void* p = 0; int e = hipMalloc(&p, n);
        uint64_t u = 0, q = 0, d = 0, pk = 0; stats_fn f = (stats_fn)dlsym(RTLD_DEFAULT, "gpushare_shim_stats");
        if (f) f(&u, &q, &d, &pk); int fe = 0; for (int k = 0; k < np; ++k) if (ptrs[k]) fe |= hipFree(ptrs[k]);
        uint64_t u2 = 0; if (f) f(&u2, &q, &d, &pk);
        printf("{\"op\":\"child\",\"err\":%d,\"used\":%llu,\"used_after_parent_frees\":%llu}\n", e,
               (unsigned long long)u, (unsigned long long)u2); fflush(stdout); _exit(0); }
      int st = 0; waitpid(c, &st, 0); ++i; printf("{\"op\":\"fork\",\"status\":%d}\n", st); }
    else if (!strcmp(argv[i], "free")) { int k = atoi(argv[++i]); int e = hipFree(ptrs[k]); ptrs[k] = 0;
      printf("{\"op\":\"free\",\"idx\":%d,\"err\":%d}\n", k, e); }
    else if (!strcmp(argv[i], "freeall")) { for (int k = 0; k < np; ++k) if (ptrs[k]) hipFree(ptrs[k]); np = 0; printf("{\"op\":\"freeall\"}\n"); }
    else if (!strcmp(argv[i], "info")) { size_t f = 0, t = 0; int e = hipMemGetInfo(&f, &t);
      printf("{\"op\":\"info\",\"free\":%zu,\"total\":%zu,\"err\":%d}\n", f, t, e); }
    else if (!strcmp(argv[i], "threads")) { int nt = atoi(argv[++i]); int it = atoi(argv[++i]); size_t n = strtoull(argv[++i], 0, 10);
      pthread_t th[64]; struct targ a[64]; int ok = 0, den = 0; if (nt > 64) nt = 64;
      for (int t = 0; t < nt; ++t) { a[t].iters = it; a[t].n = n; a[t].ok = a[t].denied = 0; pthread_create(&th[t], 0, worker, &a[t]); }
      for (int t = 0; t < nt; ++t) { pthread_join(th[t], 0); ok += a[t].ok; den += a[t].denied; }
      printf("{\"op\":\"threads\",\"ok\":%d,\"denied\":%d}\n", ok, den); }
    else if (!strcmp(argv[i], "stats")) { stats_fn f = (stats_fn)dlsym(RTLD_DEFAULT, "gpushare_shim_stats");
      uint64_t u = 0, q = 0, d = 0, pk = 0; int e = f ? f(&u, &q, &d, &pk) : -1;
      printf("{\"op\":\"stats\",\"enabled\":%d,\"used\":%llu,\"quota\":%llu,\"denied\":%llu,\"peak\":%llu}\n", e,
             (unsigned long long)u, (unsigned long long)q, (unsigned long long)d, (unsigned long long)pk); }
    else if (!strcmp(argv[i], "gem")) {   /* "gem BYTES DOMAINS": amdgpu GEM_CREATE on the render fd */
      int rfd = g_render_fd >= 0 ? g_render_fd : open("/dev/null", O_RDWR);
      struct { uint64_t size, align, domains, flags; } a = {strtoull(argv[i + 1], 0, 10), 4096, strtoull(argv[i + 2], 0, 10), 0};
      unsigned long req = ((unsigned long)3 << 30) | ((unsigned long)32 << 16) | ((unsigned long)'d' << 8) | 0x40;
      int r = ioctl(rfd, req, &a); i += 2; g_render_fd = rfd;
      printf("{\"op\":\"gem\",\"err\":%d,\"handle\":%u,\"fd\":%d}\n", r ? errno : 0, r ? 0u : *(uint32_t*)&a, rfd); }
    else if (!strcmp(argv[i], "gemclose")) { struct { uint32_t h, pad; } c = {(uint32_t)atoi(argv[++i]), 0};
      unsigned long req = ((unsigned long)1 << 30) | ((unsigned long)8 << 16) | ((unsigned long)'d' << 8) | 0x09;
      int r = ioctl(g_render_fd, req, &c); printf("{\"op\":\"gemclose\",\"err\":%d}\n", r); }
    else if (!strcmp(argv[i], "closefd")) { int fd = g_render_fd; int r = close(fd);
      g_render_fd = -1; printf("{\"op\":\"closefd\",\"err\":%d}\n", r); }
    /* DRM file identity through a synthetic /proc (GPUSHARE_SHIM_PROC_ROOT): "drmfile CID" gives
       the render fd the kernel's drm-client-id CID; "dup" duplicates it (same file, same id) */
    else if (!strcmp(argv[i], "drmfile")) { if (g_render_fd < 0) g_render_fd = open("/dev/null", O_RDWR);
      g_cid = strtoull(argv[++i], 0, 10); fake_fd(getpid(), g_render_fd, g_cid);
      printf("{\"op\":\"drmfile\",\"fd\":%d}\n", g_render_fd); }
    else if (!strcmp(argv[i], "dup")) { g_dup_fd = dup(g_render_fd); fake_fd(getpid(), g_dup_fd, g_cid);
      printf("{\"op\":\"dup\",\"fd\":%d}\n", g_dup_fd); }
    else if (!strcmp(argv[i], "swapdup")) { int t = g_render_fd; g_render_fd = g_dup_fd; g_dup_fd = t;
      printf("{\"op\":\"swapdup\"}\n"); }
    else if (!strcmp(argv[i], "closedup")) { int fd = g_dup_fd; int r = close(fd);
      g_dup_fd = -1; printf("{\"op\":\"closedup\",\"err\":%d}\n", r); }
    /* "forkhold": a child inherits the render fd and keeps it open until "killhold" */
    else if (!strcmp(argv[i], "forkhold")) { int pp[2]; if (pipe(pp)) return 9; fflush(stdout); pid_t c = fork();
      if (c == 0) { close(pp[1]); fake_fd(getpid(), g_render_fd, g_cid); char b; ssize_t n = read(pp[0], &b, 1); (void)n; _exit(0); }
      close(pp[0]); g_hold_pid = c; g_hold_pipe = pp[1]; g_hold_fd = g_render_fd;
      for (int k = 0; k < 200 && !fake_exists(c, g_render_fd); ++k) usleep(5000);
      printf("{\"op\":\"forkhold\",\"pid\":%d}\n", (int)c); }
    else if (!strcmp(argv[i], "killhold")) { close(g_hold_pipe); int st = 0; waitpid(g_hold_pid, &st, 0);
      fake_fd(g_hold_pid, g_hold_fd, 0); printf("{\"op\":\"killhold\",\"status\":%d}\n", st); }
    else if (!strcmp(argv[i], "prime")) { struct { uint32_t h, flags; int32_t fd; } a = {(uint32_t)atoi(argv[++i]), 0, -1};
      unsigned long req = ((unsigned long)3 << 30) | ((unsigned long)12 << 16) | ((unsigned long)'d' << 8) | 0x2d;
      int r = ioctl(g_render_fd, req, &a); printf("{\"op\":\"prime\",\"err\":%d,\"fd\":%d}\n", r ? errno : 0, a.fd); }
    else if (!strcmp(argv[i], "sleep")) { usleep((useconds_t)(atof(argv[++i]) * 1e6)); }
    else if (!strcmp(argv[i], "crash")) { fflush(stdout); _exit(3); }
    else if (!strcmp(argv[i], "vres")) { g_vsize = strtoull(argv[++i], 0, 10); void* b = 0;
      int e = hipMemAddressReserve(&b, g_vsize, 0, 0, 0); g_vbase = (char*)b; g_vcur = 0;
      printf("{\"op\":\"vres\",\"err\":%d,\"aligned\":%d}\n", e, (int)(((uintptr_t)b & ((1ull << 30) - 1)) == 0)); }
    else if (!strcmp(argv[i], "vpage")) { size_t n = strtoull(argv[++i], 0, 10); uint64_t h = 0;
      struct vprop pr; memset(&pr, 0, sizeof pr); pr.type = 1; pr.loc.type = 1; pr.loc.id = 0;
      int e = hipMemCreate(&h, n, &pr, 0), me = -1, ae = -1;
      if (!e) { me = hipMemMap(g_vbase + g_vcur, n, 0, h, 0);
        struct vaccess ac; memset(&ac, 0, sizeof ac); ac.loc.type = 1; ac.flags = 3;
        if (!me) { ae = hipMemSetAccess(g_vbase + g_vcur, n, &ac, 1); g_vpages[g_nv].va = g_vbase + g_vcur;
          g_vpages[g_nv].h = h; g_vpages[g_nv].n = n; g_nv++; g_vcur += n; } else hipMemRelease(h); }
      printf("{\"op\":\"vpage\",\"n\":%zu,\"err\":%d,\"map\":%d,\"access\":%d,\"idx\":%d}\n", n, e, me, ae, e || me ? -1 : g_nv - 1); }
    else if (!strcmp(argv[i], "vdrop")) { int k = atoi(argv[++i]); int ue = hipMemUnmap(g_vpages[k].va, g_vpages[k].n);
      int re = hipMemRelease(g_vpages[k].h); printf("{\"op\":\"vdrop\",\"unmap\":%d,\"release\":%d}\n", ue, re); }
    else if (!strcmp(argv[i], "vfree")) { int e = hipMemAddressFree(g_vbase, g_vsize); printf("{\"op\":\"vfree\",\"err\":%d}\n", e); }
    else if (!strcmp(argv[i], "vstats")) {
      int (*f)(uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*) =
          (int (*)(uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*))dlsym(RTLD_DEFAULT, "gpushare_shim_vmm_stats");
      uint64_t c = 0, am = 0, rp = 0, sb = 0, sn = 0; int w = f ? f(&c, &am, &rp, &sb, &sn) : -2;
      printf("{\"op\":\"vstats\",\"windows\":%d,\"creates\":%llu,\"arena_maps\":%llu,\"real_pieces\":%llu,"
             "\"slots_backed\":%llu,\"slots_now\":%llu}\n", w, (unsigned long long)c, (unsigned long long)am,
             (unsigned long long)rp, (unsigned long long)sb, (unsigned long long)sn); }
    else if (!strcmp(argv[i], "poolasync")) { size_t n = strtoull(argv[++i], 0, 10); void* pool = 0; void* p = 0;
      hipDeviceGetDefaultMemPool(&pool, 0); int e = hipMallocFromPoolAsync(&p, n, pool, 0);
      printf("{\"op\":\"poolasync\",\"n\":%zu,\"err\":%d,\"idx\":%d,\"p\":%llu}\n", n, e, e ? -1 : np,
             (unsigned long long)(uintptr_t)p); if (!e) ptrs[np++] = p; }
    else if (!strcmp(argv[i], "timefree")) { int k = atoi(argv[++i]); double t = now_ms(); int e = hipFree(ptrs[k]); ptrs[k] = 0;
      printf("{\"op\":\"timefree\",\"err\":%d,\"ms\":%.3f}\n", e, now_ms() - t); }
    else if (!strcmp(argv[i], "timealloc")) { size_t n = strtoull(argv[++i], 0, 10); void* p = 0; double t = now_ms();
      int e = hipMalloc(&p, n); printf("{\"op\":\"timealloc\",\"err\":%d,\"ms\":%.3f,\"idx\":%d,\"p\":%llu}\n", e,
      now_ms() - t, e ? -1 : np, (unsigned long long)(uintptr_t)p); if (!e) ptrs[np++] = p; }
    else if (!strcmp(argv[i], "freestats")) { int (*f)(uint64_t*, uint64_t*, uint64_t*, uint64_t*) =
        (int (*)(uint64_t*, uint64_t*, uint64_t*, uint64_t*))dlsym(RTLD_DEFAULT, "gpushare_shim_free_stats");
      uint64_t d = 0, pe = 0, w = 0, st = 0; if (f) f(&d, &pe, &w, &st);
      printf("{\"op\":\"freestats\",\"deferred\":%llu,\"pending\":%llu,\"device_waits\":%llu,\"streams\":%llu}\n",
             (unsigned long long)d, (unsigned long long)pe, (unsigned long long)w, (unsigned long long)st); }
    else if (!strcmp(argv[i], "extra")) { int (*f)(uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*) =
        (int (*)(uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t*))dlsym(RTLD_DEFAULT, "gpushare_shim_arena_extra");
      uint64_t x = 0, xd = 0, da = 0, db = 0, lim = 0; int on = f ? f(&x, &xd, &da, &db, &lim) : -2;
      printf("{\"op\":\"extra\",\"on\":%d,\"extends\":%llu,\"extended\":%llu,\"driver_allocs\":%llu,\"driver_bytes\":%llu,\"limit\":%llu}\n",
             on, (unsigned long long)x, (unsigned long long)xd, (unsigned long long)da, (unsigned long long)db, (unsigned long long)lim); }
    else if (!strcmp(argv[i], "ipcget")) { int k = atoi(argv[++i]); ipch_t h; memset(&h, 0, sizeof h);
      int e = hipIpcGetMemHandle(&h, ptrs[k]); char hex[129]; for (int j = 0; j < 64; ++j) sprintf(hex + 2 * j, "%02x", (unsigned char)h.reserved[j]);
      printf("{\"op\":\"ipcget\",\"err\":%d,\"handle\":\"%s\"}\n", e, hex); }
    else if (!strcmp(argv[i], "ipcopen")) { const char* hex = argv[++i]; ipch_t h; memset(&h, 0, sizeof h);
      for (int j = 0; j < 64 && hex[2 * j]; ++j) { unsigned v = 0; sscanf(hex + 2 * j, "%2x", &v); h.reserved[j] = (char)v; }
      void* p = 0; int e = hipIpcOpenMemHandle(&p, h, 1);
      printf("{\"op\":\"ipcopen\",\"err\":%d,\"idx\":%d,\"p\":%llu}\n", e, e ? -1 : np, (unsigned long long)(uintptr_t)p);
      if (!e) ptrs[np++] = p; }
    else if (!strcmp(argv[i], "ipcclose")) { int k = atoi(argv[++i]); int e = hipIpcCloseMemHandle(ptrs[k]); ptrs[k] = 0;
      printf("{\"op\":\"ipcclose\",\"err\":%d}\n", e); }
    else if (!strcmp(argv[i], "ipcstats")) { int (*f)(uint64_t*, uint64_t*, uint64_t*, uint64_t*) =
        (int (*)(uint64_t*, uint64_t*, uint64_t*, uint64_t*))dlsym(RTLD_DEFAULT, "gpushare_shim_ipc_stats");
      uint64_t ex = 0, sv = 0, op = 0, on = 0; if (f) f(&ex, &sv, &op, &on);
      printf("{\"op\":\"ipcstats\",\"exports\":%llu,\"served\":%llu,\"opened\":%llu,\"open_now\":%llu}\n",
             (unsigned long long)ex, (unsigned long long)sv, (unsigned long long)op, (unsigned long long)on); }
    else if (!strcmp(argv[i], "range")) { int k = atoi(argv[++i]); size_t off = strtoull(argv[++i], 0, 10); void* b = 0; size_t n = 0;
      int e = hipMemGetAddressRange(&b, &n, (char*)ptrs[k] + off);
      printf("{\"op\":\"range\",\"err\":%d,\"base\":%llu,\"size\":%zu}\n", e, (unsigned long long)(uintptr_t)b, n); }
    else if (!strcmp(argv[i], "retain")) { int k = atoi(argv[++i]); uint64_t h = 0; int e = hipMemRetainAllocationHandle(&h, ptrs[k]);
      printf("{\"op\":\"retain\",\"err\":%d}\n", e); }
    else if (!strcmp(argv[i], "forksleep")) { int ms = atoi(argv[++i]); fflush(stdout); pid_t c = fork();
      if (c == 0) { usleep((useconds_t)ms * 1000); _exit(0); }
      printf("{\"op\":\"forksleep\",\"pid\":%d}\n", (int)c); }
    else if (!strcmp(argv[i], "sigterm_handler")) { signal(SIGTERM, on_term); printf("{\"op\":\"sigterm_handler\"}\n"); }
    else if (!strcmp(argv[i], "wait")) { fflush(stdout); char b[256]; while (read(0, b, sizeof b) > 0) {} }  /* until stdin closes */
    fflush(stdout);
  }
  return 0;
}
