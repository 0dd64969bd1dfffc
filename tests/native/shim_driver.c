// Test driver: executes allocation commands against the (stub or real) HIP runtime and
// prints one JSON line per command. Linked against libamdhip64.so.7 like any HIP program.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
typedef int hipError_t;
hipError_t hipMalloc(void**, size_t); hipError_t hipFree(void*);
hipError_t hipMemGetInfo(size_t*, size_t*); hipError_t hipMallocAsync(void**, size_t, void*);
hipError_t hipFreeAsync(void*, void*); hipError_t hipMemCreate(uint64_t*, size_t, const void*, unsigned long long);
hipError_t hipMemRelease(uint64_t);
int main(int argc, char** argv) {
  void* ptrs[4096]; int np = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "alloc")) { size_t n = strtoull(argv[++i], 0, 10); void* p = 0; int e = hipMalloc(&p, n);
      printf("{\"op\":\"alloc\",\"n\":%zu,\"err\":%d,\"idx\":%d}\n", n, e, e ? -1 : np); if (!e) ptrs[np++] = p; }
    else if (!strcmp(argv[i], "async")) { size_t n = strtoull(argv[++i], 0, 10); void* p = 0; int e = hipMallocAsync(&p, n, 0);
      printf("{\"op\":\"async\",\"n\":%zu,\"err\":%d,\"idx\":%d}\n", n, e, e ? -1 : np); if (!e) ptrs[np++] = p; }
    else if (!strcmp(argv[i], "vmm")) { size_t n = strtoull(argv[++i], 0, 10); uint64_t h = 0; int e = hipMemCreate(&h, n, 0, 0);
      printf("{\"op\":\"vmm\",\"n\":%zu,\"err\":%d}\n", n, e); if (!e) hipMemRelease(h); }
    else if (!strcmp(argv[i], "free")) { int k = atoi(argv[++i]); int e = hipFree(ptrs[k]); ptrs[k] = 0;
      printf("{\"op\":\"free\",\"idx\":%d,\"err\":%d}\n", k, e); }
    else if (!strcmp(argv[i], "freeall")) { for (int k = 0; k < np; ++k) if (ptrs[k]) hipFree(ptrs[k]); np = 0; printf("{\"op\":\"freeall\"}\n"); }
    else if (!strcmp(argv[i], "info")) { size_t f = 0, t = 0; int e = hipMemGetInfo(&f, &t);
      printf("{\"op\":\"info\",\"free\":%zu,\"total\":%zu,\"err\":%d}\n", f, t, e); }
    else if (!strcmp(argv[i], "sleep")) { usleep((useconds_t)(atof(argv[++i]) * 1e6)); }
    else if (!strcmp(argv[i], "crash")) { fflush(stdout); _exit(3); }
    fflush(stdout);
  }
  return 0;
}
