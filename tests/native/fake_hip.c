// Stub HIP runtime for CPU-only tests of the quota shim: host malloc stands in for HBM.
// Exposes the exact entry points libgpushare_hipquota.so interposes (same soname as ROCm).
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
typedef int hipError_t;
static size_t g_total = (size_t)16 << 30, g_used = 0;
// g_used is updated atomically: the threaded driver command allocates from many threads.
static void* take(size_t n) { char* p = malloc(16); if (!p) return 0; *(size_t*)p = n; return p + 8; }
hipError_t hipMalloc(void** p, size_t n) {
  size_t cur = __atomic_load_n(&g_used, __ATOMIC_RELAXED);
  do { if (cur + n > g_total) return 2; } while (!__atomic_compare_exchange_n(&g_used, &cur, cur + n, 1, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED));
  *p = take(n); return 0; }
hipError_t hipExtMallocWithFlags(void** p, size_t n, unsigned f) { return hipMalloc(p, n); }
hipError_t hipMallocManaged(void** p, size_t n, unsigned f) { return hipMalloc(p, n); }
hipError_t hipMallocAsync(void** p, size_t n, void* s) { return hipMalloc(p, n); }
hipError_t hipFree(void* p) { if (p) { char* b = (char*)p - 8; __atomic_fetch_sub(&g_used, *(size_t*)b, __ATOMIC_ACQ_REL); free(b); } return 0; }
hipError_t hipFreeAsync(void* p, void* s) { return hipFree(p); }
hipError_t hipMemGetInfo(size_t* f, size_t* t) { *f = g_total - __atomic_load_n(&g_used, __ATOMIC_ACQUIRE); *t = g_total; return 0; }
hipError_t hipDeviceTotalMem(size_t* b, int d) { *b = g_total; return 0; }
hipError_t hipMemCreate(uint64_t* h, size_t n, const void* prop, unsigned long long fl) { void* p; int e = hipMalloc(&p, n); *h = (uint64_t)p; return e; }
hipError_t hipMemRelease(uint64_t h) { return hipFree((void*)h); }
