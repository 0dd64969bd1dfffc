/* dlsym for libgpushare_comgrcache.so (comgr_action_cache.cpp). A lookup of
 * "amd_comgr_do_action" in a library handle gets the caching wrapper; every other lookup is a
 * guaranteed tail call into the C library's dlsym, so the return address glibc reads to find the
 * caller (RTLD_NEXT, namespaces) is still the real caller's. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <string.h>

typedef void* (*gs_dlsym_fn)(void*, const char*);
void* gs_comgr_wrap(void* handle);
gs_dlsym_fn gs_comgr_real_dlsym(void);

__attribute__((visibility("default"))) void* dlsym(void* restrict handle, const char* restrict name) {
  if (__builtin_expect(name[0] == 'a', 0) && handle != RTLD_NEXT && strcmp(name, "amd_comgr_do_action") == 0) {
    void* w = gs_comgr_wrap(handle);
    if (w) return w;
  }
  gs_dlsym_fn real = gs_comgr_real_dlsym();
  __attribute__((musttail)) return real(handle, name);
}
