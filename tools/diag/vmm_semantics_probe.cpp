// VMM semantics the quota shim's arena depends on, probed on whichever HIP runtime the process
// loaded (symbols from dlsym(RTLD_DEFAULT)): PyTorch's bundled runtime when loaded from Python
// after `import torch` (tools/diag/vmm_semantics_probe.py), the system runtime when built as an
// executable linked with -lamdhip64.
//
//   g++ -std=c++17 -O1 -shared -fPIC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
//       -o tools/diag/build/libvmm_semantics_probe.so tools/diag/vmm_semantics_probe.cpp -ldl
//   g++ -std=c++17 -O1 -DPROBE_MAIN -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
//       -o tools/diag/build/vmm_semantics_probe tools/diag/vmm_semantics_probe.cpp \
//       -L/opt/rocm/lib -lamdhip64 -ldl -Wl,-rpath,/opt/rocm/lib
//
// Questions (each answered by an error code and, where it maps, by a read-back of bytes):
//   same_handle_two_vas  one physical handle mapped at two VAs at once: do they alias?
//   map_sub_size         hipMemMap of fewer bytes than the handle holds (offset 0)
//   map_offset           hipMemMap at a non-zero offset into the handle
//   imported_two_vas     the same for a handle imported from the handle's own dma-buf fd
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <link.h>

#include <cstring>

namespace {
// the libamdhip64 this process has loaded (PyTorch loads its own copy RTLD_LOCAL: RTLD_DEFAULT
// does not see it), else the system's
void* hip_lib() {
  static void* h = nullptr;
  if (h) return h;
  const char* path = nullptr;
  dl_iterate_phdr(
      [](dl_phdr_info* info, size_t, void* data) {
        if (info->dlpi_name && std::strstr(info->dlpi_name, "libamdhip64.so")) {
          *static_cast<const char**>(data) = info->dlpi_name;
          return 1;
        }
        return 0;
      },
      &path);
  if (path) h = dlopen(path, RTLD_NOLOAD | RTLD_LAZY);
  if (!h) h = dlopen("libamdhip64.so.7", RTLD_LAZY);
  return h;
}

template <class F>
F sym(const char* n) {
  void* h = hip_lib();
  return reinterpret_cast<F>(h ? dlsym(h, n) : nullptr);
}

struct Api {
  decltype(&hipSetDevice) setdev = sym<decltype(&hipSetDevice)>("hipSetDevice");
  decltype(&hipMemCreate) create = sym<decltype(&hipMemCreate)>("hipMemCreate");
  decltype(&hipMemRelease) release = sym<decltype(&hipMemRelease)>("hipMemRelease");
  decltype(&hipMemAddressReserve) reserve = sym<decltype(&hipMemAddressReserve)>("hipMemAddressReserve");
  decltype(&hipMemAddressFree) vfree = sym<decltype(&hipMemAddressFree)>("hipMemAddressFree");
  decltype(&hipMemMap) map = sym<decltype(&hipMemMap)>("hipMemMap");
  decltype(&hipMemUnmap) unmap = sym<decltype(&hipMemUnmap)>("hipMemUnmap");
  decltype(&hipMemSetAccess) access = sym<decltype(&hipMemSetAccess)>("hipMemSetAccess");
  decltype(&hipMemset) memset_ = sym<decltype(&hipMemset)>("hipMemset");
  decltype(&hipMemcpy) memcpy_ = sym<decltype(&hipMemcpy)>("hipMemcpy");
  decltype(&hipDeviceSynchronize) sync = sym<decltype(&hipDeviceSynchronize)>("hipDeviceSynchronize");
  decltype(&hipRuntimeGetVersion) version = sym<decltype(&hipRuntimeGetVersion)>("hipRuntimeGetVersion");
  decltype(&hipMemExportToShareableHandle) exp =
      sym<decltype(&hipMemExportToShareableHandle)>("hipMemExportToShareableHandle");
  decltype(&hipMemImportFromShareableHandle) imp =
      sym<decltype(&hipMemImportFromShareableHandle)>("hipMemImportFromShareableHandle");
  decltype(&hipGetLastError) lasterr = sym<decltype(&hipGetLastError)>("hipGetLastError");
};

std::string out;
void rec(const char* k, int v) {
  char b[128];
  std::snprintf(b, sizeof b, "%s\"%s\": %d", out.size() > 1 ? ", " : "", k, v);
  out += b;
}

bool set_rw(Api& A, void* p, size_t n) {
  hipMemAccessDesc d;
  std::memset(&d, 0, sizeof d);
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  return A.access(p, n, &d, 1) == hipSuccess;
}

// 1 = bytes written through `a` read back through `b`, 0 = not, -1 = could not check
int alias(Api& A, char* a, char* b, size_t off) {
  if (A.memset_(a + off, 0x5a, 4096) != hipSuccess) return -1;
  A.sync();
  unsigned char host[4096];
  if (A.memcpy_(host, b, 4096, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  for (unsigned char c : host)
    if (c != 0x5a) return 0;
  return 1;
}
}  // namespace

extern "C" const char* vmm_semantics_probe(unsigned long long gran_mib) {
  Api A;
  out = "{";
  if (!A.create || !A.map) {
    out += "\"error\": \"no HIP VMM entry points in this process\"}";
    return out.c_str();
  }
  int ver = 0;
  if (A.version) (void)A.version(&ver);
  rec("runtime_version", ver);
  A.setdev(0);
  size_t gran = size_t(gran_mib) << 20, page = 20ull << 20;
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof p);
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  hipMemGenericAllocationHandle_t h = nullptr;
  rec("create", A.create(&h, gran, &p, 0));
  void *va1 = nullptr, *va2 = nullptr, *va3 = nullptr;
  rec("reserve1", A.reserve(&va1, gran, 0, nullptr, 0));
  rec("reserve2", A.reserve(&va2, gran, 0, nullptr, 0));
  rec("reserve3", A.reserve(&va3, 4 * page, 0, nullptr, 0));
  int e = A.map(va1, gran, 0, h, 0);
  rec("map_first", e);
  rec("access_first", set_rw(A, va1, gran));
  e = A.map(va2, gran, 0, h, 0);
  rec("same_handle_two_vas", e);
  if (e == hipSuccess) {
    rec("access_second", set_rw(A, va2, gran));
    rec("same_handle_two_vas_alias", alias(A, static_cast<char*>(va1), static_cast<char*>(va2), 0));
    rec("unmap_second", A.unmap(va2, gran));
  }
  A.lasterr();
  e = A.map(va3, page, 0, h, 0);
  rec("map_sub_size", e);
  if (e == hipSuccess) {
    rec("access_sub", set_rw(A, va3, page));
    rec("map_sub_size_alias", alias(A, static_cast<char*>(va1), static_cast<char*>(va3), 0));
    rec("unmap_sub", A.unmap(va3, page));
  }
  A.lasterr();
  e = A.map(static_cast<char*>(va3) + page, page, 2 * page, h, 0);
  rec("map_offset", e);
  if (e == hipSuccess) {
    rec("access_offset", set_rw(A, static_cast<char*>(va3) + page, page));
    rec("map_offset_alias", alias(A, static_cast<char*>(va1), static_cast<char*>(va3) + page, 2 * page));
    rec("unmap_offset", A.unmap(static_cast<char*>(va3) + page, page));
  }
  A.lasterr();
  // an imported handle (what the shim holds): a second mapping of it
  int fd = -1;
  if (A.exp && A.imp && A.exp(&fd, h, hipMemHandleTypePosixFileDescriptor, 0) == hipSuccess && fd >= 0) {
    hipMemGenericAllocationHandle_t hi = nullptr;
    e = A.imp(&hi, &fd, hipMemHandleTypePosixFileDescriptor);
    if (e == hipErrorInvalidValue) e = A.imp(&hi, reinterpret_cast<void*>(static_cast<intptr_t>(fd)), hipMemHandleTypePosixFileDescriptor);
    rec("import", e);
    if (e == hipSuccess) {
      e = A.map(va2, gran, 0, hi, 0);
      rec("imported_two_vas", e);
      if (e == hipSuccess) {
        rec("imported_access", set_rw(A, va2, gran));
        rec("imported_two_vas_alias", alias(A, static_cast<char*>(va1), static_cast<char*>(va2), 4096));
        rec("imported_unmap", A.unmap(va2, gran));
      }
      A.lasterr();
      e = A.map(va3, page, 0, hi, 0);
      rec("imported_sub_size", e);
      if (e == hipSuccess) A.unmap(va3, page);
      A.lasterr();
      e = A.map(static_cast<char*>(va3) + page, page, page, hi, 0);
      rec("imported_offset", e);
      if (e == hipSuccess) {
        rec("imported_offset_access", set_rw(A, static_cast<char*>(va3) + page, page));
        rec("imported_offset_alias", alias(A, static_cast<char*>(va1), static_cast<char*>(va3) + page, page));
        A.unmap(static_cast<char*>(va3) + page, page);
      }
      A.lasterr();
      rec("imported_release", A.release(hi));
    }
    close(fd);
  }
  rec("unmap_first", A.unmap(va1, gran));
  rec("release", A.release(h));
  A.vfree(va1, gran);
  A.vfree(va2, gran);
  A.vfree(va3, 4 * page);
  out += "}";
  return out.c_str();
}

#ifdef PROBE_MAIN
int main(int argc, char** argv) {
  std::puts(vmm_semantics_probe(argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024));
  return 0;
}
#endif
