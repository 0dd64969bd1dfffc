// gpushare-comgr-probe: the compile the HIP runtime does for its blit kernels at a process's first
// stream, without a GPU: OpenCL source -> bitcode with the device libraries -> link -> codegen ->
// executable for gfx950, through comgr loaded the way the runtime loads it (dlopen + dlsym of each
// entry point). tests/test_comgr_action_cache.py runs it with and without
// libgpushare_comgrcache.so preloaded. Prints one JSON line: per-step ms, the executable's size
// and a digest of its bytes, and the cache's counters when the library is loaded.
#include <amd_comgr/amd_comgr.h>
#include <dlfcn.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

static const char kSource[] = R"CL(
__kernel void gs_probe_fill(__global uint4* dst, uint4 v, ulong n) {
  for (ulong i = get_global_id(0); i < n; i += get_global_size(0)) dst[i] = v;
}
__kernel void gs_probe_copy(__global const uint4* src, __global uint4* dst, ulong n) {
  for (ulong i = get_global_id(0); i < n; i += get_global_size(0)) dst[i] = src[i];
}
)CL";

#define SYM(name) auto name##_ = reinterpret_cast<decltype(&name)>(dlsym(h, #name))

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const char* variant = argc > 1 ? argv[1] : "";   // a different source = a different key
  bool logging = argc > 2 && argv[2][0] == '1';     // as the HIP runtime does: a LOG object per result
  void* h = dlopen("libamd_comgr.so.3", RTLD_NOW | RTLD_LOCAL);
  if (h == nullptr) {
    std::printf("{\"ok\": false, \"error\": \"dlopen: %s\"}\n", dlerror());
    return 2;
  }
  SYM(amd_comgr_do_action);
  SYM(amd_comgr_create_data);
  SYM(amd_comgr_set_data);
  SYM(amd_comgr_set_data_name);
  SYM(amd_comgr_create_data_set);
  SYM(amd_comgr_destroy_data_set);
  SYM(amd_comgr_data_set_add);
  SYM(amd_comgr_release_data);
  SYM(amd_comgr_create_action_info);
  SYM(amd_comgr_destroy_action_info);
  SYM(amd_comgr_action_info_set_isa_name);
  SYM(amd_comgr_action_info_set_language);
  SYM(amd_comgr_action_info_set_option_list);
  SYM(amd_comgr_action_info_set_logging);
  SYM(amd_comgr_action_data_get_data);
  SYM(amd_comgr_get_data);
  if (!amd_comgr_do_action_ || !amd_comgr_get_data_) {
    std::printf("{\"ok\": false, \"error\": \"dlsym\"}\n");
    return 2;
  }
  std::string src = std::string(kSource) + "// " + variant + "\n";
  amd_comgr_data_t source;
  amd_comgr_data_set_t in, bc, linked, reloc, exe;
  amd_comgr_action_info_t info;
  amd_comgr_create_data_(AMD_COMGR_DATA_KIND_SOURCE, &source);
  amd_comgr_set_data_(source, src.size(), src.data());
  amd_comgr_set_data_name_(source, "gs_probe.cl");
  amd_comgr_create_data_set_(&in);
  amd_comgr_data_set_add_(in, source);
  amd_comgr_create_data_set_(&bc);
  amd_comgr_create_data_set_(&linked);
  amd_comgr_create_data_set_(&reloc);
  amd_comgr_create_data_set_(&exe);
  amd_comgr_create_action_info_(&info);
  amd_comgr_action_info_set_isa_name_(info, "amdgcn-amd-amdhsa--gfx950");
  amd_comgr_action_info_set_language_(info, AMD_COMGR_LANGUAGE_OPENCL_1_2);
  const char* opts[] = {"-O3", "-cl-std=CL1.2", "-cl-kernel-arg-info"};
  amd_comgr_action_info_set_option_list_(info, opts, 3);
  if (logging) amd_comgr_action_info_set_logging_(info, true);
  double t[5];
  amd_comgr_status_t st[4];
  t[0] = now_ms();
  st[0] = amd_comgr_do_action_(AMD_COMGR_ACTION_COMPILE_SOURCE_WITH_DEVICE_LIBS_TO_BC, info, in, bc);
  t[1] = now_ms();
  st[1] = amd_comgr_do_action_(AMD_COMGR_ACTION_LINK_BC_TO_BC, info, bc, linked);
  t[2] = now_ms();
  st[2] = amd_comgr_do_action_(AMD_COMGR_ACTION_CODEGEN_BC_TO_RELOCATABLE, info, linked, reloc);
  t[3] = now_ms();
  st[3] = amd_comgr_do_action_(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, info, reloc, exe);
  t[4] = now_ms();
  for (int i = 0; i < 4; ++i) {
    if (st[i] != AMD_COMGR_STATUS_SUCCESS) {
      std::printf("{\"ok\": false, \"error\": \"step %d status %d\"}\n", i, int(st[i]));
      return 1;
    }
  }
  amd_comgr_data_t obj;
  size_t n = 0;
  std::string bytes;
  if (amd_comgr_action_data_get_data_(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, 0, &obj) != AMD_COMGR_STATUS_SUCCESS ||
      amd_comgr_get_data_(obj, &n, nullptr) != AMD_COMGR_STATUS_SUCCESS) {
    std::printf("{\"ok\": false, \"error\": \"no executable\"}\n");
    return 1;
  }
  bytes.resize(n);
  amd_comgr_get_data_(obj, &n, &bytes[0]);
  amd_comgr_release_data_(obj);
  uint64_t d = 1469598103934665603ull;   // FNV-1a of the executable
  for (unsigned char c : bytes) d = (d ^ c) * 1099511628211ull;
  uint64_t s[5] = {0, 0, 0, 0, 0};
  auto stats = reinterpret_cast<int (*)(uint64_t*, int)>(dlsym(RTLD_DEFAULT, "gpushare_comgr_cache_stats"));
  int ns = stats ? stats(s, 5) : 0;
  std::printf("{\"ok\": true, \"compile_ms\": %.3f, \"link_bc_ms\": %.3f, \"codegen_ms\": %.3f, \"link_exe_ms\": %.3f, "
              "\"total_ms\": %.3f, \"exe_bytes\": %zu, \"exe_digest\": \"%016llx\", \"cache\": %s",
              t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3], t[4] - t[0], n, (unsigned long long)d,
              ns ? "{" : "null");
  if (ns)
    std::printf("\"hits\": %llu, \"misses\": %llu, \"stores\": %llu, \"bypassed\": %llu, \"errors\": %llu}",
                (unsigned long long)s[0], (unsigned long long)s[1], (unsigned long long)s[2],
                (unsigned long long)s[3], (unsigned long long)s[4]);
  std::printf("}\n");
  amd_comgr_destroy_action_info_(info);
  amd_comgr_release_data_(source);
  amd_comgr_destroy_data_set_(in);
  amd_comgr_destroy_data_set_(bc);
  amd_comgr_destroy_data_set_(linked);
  amd_comgr_destroy_data_set_(reloc);
  amd_comgr_destroy_data_set_(exe);
  return 0;
}
