// Who keeps a broker granule's dma-buf referenced after a tenant released it, and what does a
// tenant's first import + map cost?
//
// The HBM broker lends a granule again only when no reference to its dma-buf is left outside the
// broker (fdinfo "count"). Round 5 measured, with the quota shim under PyTorch: after the tenant's
// hipMemUnmap + hipMemRelease of its imported handles the references stay until the tenant's
// process is torn down, so a replacement pod waits for that teardown. This probe follows the
// count through one import: a child process exports 1 GiB handles and sends the fds
// (SCM_RIGHTS), as the broker does, and stays alive; this process imports one, as a tenant does:
//
//   c0  received fd only              c3  after hipMemUnmap
//   c1  after the import              c4  after hipMemRelease of the imported handle
//   c2  after map + access + memset   c5  after hipDeviceSynchronize (and 300 ms later)
//   then, on every render-node fd of this process, DRM_IOCTL_PRIME_FD_TO_HANDLE of the dma-buf and
//   DRM_IOCTL_GEM_CLOSE of the handle it names: c6 after those closes
//
// and times the first map in the process against a second granule's import / map / access.
// "warm": a hipMalloc + hipMemset + sync first, so the runtime's own one-time device work is done
// before the first map.
//
// Every HIP entry point is looked up in the libamdhip64 this process loaded: the system runtime
// when built as an executable (PROBE_MAIN, linked with -lamdhip64), PyTorch's bundled runtime
// when loaded from Python after `import torch` (tools/diag/dmabuf_ref_probe.py).
//
//   g++ -std=c++17 -O1 -DPROBE_MAIN -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o tools/diag/build/dmabuf_ref_probe
//       tools/diag/dmabuf_ref_probe.cpp -L/opt/rocm/lib -lamdhip64 -ldl -Wl,-rpath,/opt/rocm/lib
//   g++ -std=c++17 -O1 -shared -fPIC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include
//       -o tools/diag/build/libdmabuf_ref_probe.so tools/diag/dmabuf_ref_probe.cpp -ldl
#include <dirent.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <link.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {
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
#define H(name) (sym<decltype(&name)>(#name))

struct drm_prime_handle_ {
  uint32_t handle;
  uint32_t flags;
  int32_t fd;
};
struct drm_gem_close_ {
  uint32_t handle;
  uint32_t pad;
};
constexpr unsigned long kPrimeFdToHandle = _IOWR('d', 0x2e, drm_prime_handle_);
constexpr unsigned long kGemClose = _IOW('d', 0x09, drm_gem_close_);
constexpr size_t kGran = 1ull << 30;
constexpr int kFds = 5;

long now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return long(t.tv_sec) * 1000000 + t.tv_nsec / 1000;
}

int count_of(int fd) {
  char path[64];
  std::snprintf(path, sizeof path, "/proc/self/fdinfo/%d", fd);
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  char line[256];
  int c = -1;
  while (std::fgets(line, sizeof line, f))
    if (std::sscanf(line, "count: %d", &c) == 1) break;
  std::fclose(f);
  return c;
}

std::vector<int> render_fds() {
  std::vector<int> out;
  DIR* d = opendir("/proc/self/fd");
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    char link[256], path[300];
    std::snprintf(path, sizeof path, "/proc/self/fd/%s", e->d_name);
    ssize_t n = readlink(path, link, sizeof link - 1);
    if (n <= 0) continue;
    link[n] = 0;
    if (std::strstr(link, "/dev/dri/renderD")) out.push_back(std::atoi(e->d_name));
  }
  closedir(d);
  return out;
}

// other fds of this process on the same file as `fd` (the runtime's own copies)
std::vector<int> same_file_fds(int fd) {
  std::vector<int> out;
  struct stat a;
  if (fstat(fd, &a)) return out;
  DIR* d = opendir("/proc/self/fd");
  if (!d) return out;
  int self = dirfd(d);
  while (dirent* e = readdir(d)) {
    int f = std::atoi(e->d_name);
    if (e->d_name[0] < '0' || e->d_name[0] > '9' || f == fd || f == self) continue;
    struct stat b;
    if (fstat(f, &b) == 0 && b.st_dev == a.st_dev && b.st_ino == a.st_ino) out.push_back(f);
  }
  closedir(d);
  return out;
}

void send_fd(int s, int fd) {
  char b = 'f';
  iovec io{&b, 1};
  alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int))];
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  cmsghdr* c = CMSG_FIRSTHDR(&m);
  c->cmsg_level = SOL_SOCKET;
  c->cmsg_type = SCM_RIGHTS;
  c->cmsg_len = CMSG_LEN(sizeof(int));
  std::memcpy(CMSG_DATA(c), &fd, sizeof fd);
  (void)sendmsg(s, &m, 0);
}

int recv_fd(int s) {
  char b;
  iovec io{&b, 1};
  alignas(cmsghdr) char ctl[CMSG_SPACE(sizeof(int))];
  msghdr m{};
  m.msg_iov = &io;
  m.msg_iovlen = 1;
  m.msg_control = ctl;
  m.msg_controllen = sizeof ctl;
  if (recvmsg(s, &m, 0) != 1) return -1;
  cmsghdr* c = CMSG_FIRSTHDR(&m);
  int fd = -1;
  if (c && c->cmsg_type == SCM_RIGHTS) std::memcpy(&fd, CMSG_DATA(c), sizeof fd);
  return fd;
}

hipMemAllocationProp shareable() {
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof p);
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  return p;
}

// ---- the runtime's KFD ioctls (this file's ioctl interposes libc's: in the executable, or in the
// library when it is LD_PRELOADed) ----
struct KRec {
  unsigned nr;
  uint64_t handle;
  uint32_t gpu_id;
  ino_t ino;
  int kfd;
  int rc;
};
KRec g_k[8192];
int g_nk = 0;
bool g_recording = false;

constexpr unsigned long kfd_iowr(unsigned nr, unsigned size) {
  return (3ul << 30) | ((unsigned long)size << 16) | ((unsigned long)'K' << 8) | nr;
}
constexpr unsigned long kfd_iow(unsigned nr, unsigned size) {
  return (1ul << 30) | ((unsigned long)size << 16) | ((unsigned long)'K' << 8) | nr;
}
struct UnmapArgs {
  uint64_t handle, device_ids_array_ptr;
  uint32_t n_devices, n_success;
};
struct ImportArgs {
  uint64_t va_addr, handle;
  uint32_t gpu_id, dmabuf_fd;
};

ino_t ino_of(int fd) {
  struct stat st;
  return fstat(fd, &st) == 0 ? st.st_ino : 0;
}

std::string out;
void rec(const char* k, long v) { out += std::string(out.size() > 1 ? ", \"" : "\"") + k + "\": " + std::to_string(v); }

hipError_t import_fd(int rt, hipMemGenericAllocationHandle_t* h, int& fd) {
  return rt < 70100000 ? H(hipMemImportFromShareableHandle)(h, &fd, hipMemHandleTypePosixFileDescriptor)
                       : H(hipMemImportFromShareableHandle)(h, reinterpret_cast<void*>(static_cast<intptr_t>(fd)),
                                                            hipMemHandleTypePosixFileDescriptor);
}
// free the KFD objects the runtime made when it imported `fd` and has not freed: unmap them from
// their GPU, then free them. Returns how many were freed (-1: none found)
int free_leaked_imports(int fd, const char* tag) {
  ino_t ino = ino_of(fd);
  int freed = -1;
  for (int i = 0; i < g_nk; ++i) {
    if (g_k[i].nr != 0x1D || g_k[i].rc != 0 || g_k[i].ino != ino) continue;
    bool gone = false;
    for (int j = i + 1; j < g_nk; ++j) gone |= g_k[j].nr == 0x17 && g_k[j].handle == g_k[i].handle && g_k[j].rc == 0;
    if (gone) continue;
    if (freed < 0) freed = 0;
    uint32_t dev = g_k[i].gpu_id;
    UnmapArgs u{g_k[i].handle, reinterpret_cast<uint64_t>(&dev), 1, 0};
    int ru = ioctl(g_k[i].kfd, kfd_iowr(0x19, sizeof(UnmapArgs)), &u);
    uint64_t h = g_k[i].handle;
    int rf = ioctl(g_k[i].kfd, kfd_iow(0x17, sizeof(uint64_t)), &h);
    std::string k = std::string(tag) + "_unmap_rc";
    rec(k.c_str(), ru);
    k = std::string(tag) + "_free_rc";
    rec(k.c_str(), rf);
    freed += rf == 0;
  }
  return freed;
}
}  // namespace

extern "C" int ioctl(int fd, unsigned long req, ...) {
  va_list ap;
  va_start(ap, req);
  void* arg = va_arg(ap, void*);
  va_end(ap);
  static auto real = reinterpret_cast<int (*)(int, unsigned long, void*)>(dlsym(RTLD_NEXT, "ioctl"));
  int rc = real(fd, req, arg);
  unsigned nr = req & 0xff;
  if (g_recording && ((req >> 8) & 0xff) == 'K' && g_nk < 8192 &&
      (nr == 0x16 || nr == 0x17 || nr == 0x18 || nr == 0x19 || nr == 0x1D)) {
    KRec& r = g_k[g_nk++];
    r = KRec{nr, *static_cast<uint64_t*>(arg), 0, 0, fd, rc};
    if (nr == 0x1D) {
      auto* a = static_cast<ImportArgs*>(arg);
      r.handle = a->handle;
      r.gpu_id = a->gpu_id;
      r.ino = ino_of(int(a->dmabuf_fd));
    }
  }
  return rc;
}

extern "C" const char* dmabuf_ref_probe(int warm) {
  out = "{";
  if (!H(hipMemMap)) return "{\"error\": \"no HIP runtime in this process\"}";
  int sp[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sp)) return "{\"error\": \"socketpair\"}";
  pid_t child = fork();  // before this process's first HIP call
  if (child == 0) {      // the exporter (the broker's part)
    close(sp[0]);
    auto p = shareable();
    hipMemGenericAllocationHandle_t h[kFds] = {};
    int efd[kFds];
    if (H(hipSetDevice)(0) != hipSuccess) _exit(3);
    for (int i = 0; i < kFds; ++i)
      if (H(hipMemCreate)(&h[i], kGran, &p, 0) != hipSuccess ||
          H(hipMemExportToShareableHandle)(&efd[i], h[i], hipMemHandleTypePosixFileDescriptor, 0) != hipSuccess)
        _exit(3);
    for (int i = 0; i < kFds; ++i) send_fd(sp[1], efd[i]);
    char b;
    if (read(sp[1], &b, 1) < 0) _exit(4);  // until the tenant is done
    _exit(0);
  }
  close(sp[1]);
  int fds[kFds];
  for (int i = 0; i < kFds; ++i)
    if ((fds[i] = recv_fd(sp[0])) < 0) return "{\"error\": \"no fds\"}";
  int fd = fds[0], fd2 = fds[1];
  (void)H(hipSetDevice)(0);
  int rt = 0;
  (void)H(hipRuntimeGetVersion)(&rt);
  rec("runtime_version", rt);
  rec("warm", warm);
  if (warm) {  // bit 0: a hipMalloc first; bit 1: a hipMemset + sync on it as well
    void* m = nullptr;
    long t = now_us();
    rec("warm_malloc", sym<hipError_t (*)(void**, size_t)>("hipMalloc")(&m, 64 << 20));
    rec("warm_malloc_us", now_us() - t);
    if (warm & 2) {
      long t2 = now_us();
      rec("warm_memset", sym<hipError_t (*)(void*, int, size_t)>("hipMemset")(m, 0, 64 << 20));
      rec("warm_sync", H(hipDeviceSynchronize)());
      rec("warm_memset_us", now_us() - t2);
    }
    rec("warm_us", now_us() - t);
    (void)H(hipFree)(m);
  }
  hipMemAccessDesc d;
  std::memset(&d, 0, sizeof d);
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  hipMemGenericAllocationHandle_t hi = nullptr;
  g_recording = true;
  rec("c0", count_of(fd));
  long t = now_us();
  rec("import", import_fd(rt, &hi, fd));
  rec("first_import_us", now_us() - t);
  rec("c1", count_of(fd));
  void* va = nullptr;
  rec("reserve", H(hipMemAddressReserve)(&va, kGran, 0, nullptr, 0));
  t = now_us();
  rec("map", H(hipMemMap)(va, kGran, 0, hi, 0));
  rec("first_map_us", now_us() - t);
  t = now_us();
  rec("access", H(hipMemSetAccess)(va, kGran, &d, 1));
  rec("first_access_us", now_us() - t);
  rec("memset", sym<hipError_t (*)(void*, int, size_t)>("hipMemset")(va, 0, 4096));
  rec("sync0", H(hipDeviceSynchronize)());
  rec("c2", count_of(fd));
  rec("unmap", H(hipMemUnmap)(va, kGran));
  rec("c3", count_of(fd));
  rec("release_imported", H(hipMemRelease)(hi));
  rec("c4", count_of(fd));
  rec("sync", H(hipDeviceSynchronize)());
  rec("c5", count_of(fd));
  {
    // does the runtime keep a copy of the fd? (checked again for case B below, then closed)
    std::vector<int> dups = same_file_fds(fd);
    rec("dup_fds_after_release", long(dups.size()));
  }
  {
    int c = count_of(fd), ms = 0;
    while (ms < 300 && count_of(fd) == c) {
      usleep(1000);
      ++ms;
    }
    rec("c5_after_wait", count_of(fd));
    rec("c5_wait_ms", ms);
  }
  {  // a second granule into a fresh range
    hipMemGenericAllocationHandle_t h2 = nullptr;
    void* va2 = nullptr;
    t = now_us();
    rec("second_import", import_fd(rt, &h2, fd2));
    rec("second_import_us", now_us() - t);
    (void)H(hipMemAddressReserve)(&va2, kGran, 0, nullptr, 0);
    t = now_us();
    rec("second_map", H(hipMemMap)(va2, kGran, 0, h2, 0));
    rec("second_map_us", now_us() - t);
    t = now_us();
    rec("second_access", H(hipMemSetAccess)(va2, kGran, &d, 1));
    rec("second_access_us", now_us() - t);
    rec("c2_second", count_of(fd2));
    (void)H(hipMemUnmap)(va2, kGran);
    (void)H(hipMemRelease)(h2);
    (void)H(hipMemAddressFree)(va2, kGran);
    rec("c4_second", count_of(fd2));
  }
  {  // B: import, release, no map
    hipMemGenericAllocationHandle_t hb = nullptr;
    rec("b_c0", count_of(fds[2]));
    rec("b_import", import_fd(rt, &hb, fds[2]));
    rec("b_c1", count_of(fds[2]));
    rec("b_dups_while_imported", long(same_file_fds(fds[2]).size()));
    rec("b_release", H(hipMemRelease)(hb));
    rec("b_c4", count_of(fds[2]));
    std::vector<int> dups = same_file_fds(fds[2]);
    rec("b_dups_after_release", long(dups.size()));
    for (int f : dups) close(f);
    rec("b_c_after_closing_dups", count_of(fds[2]));
    rec("b_leaked_freed", free_leaked_imports(fds[2], "b"));
    rec("b_c_after_kfd_free", count_of(fds[2]));
  }
  {  // C: the full cycle, then a second release of the same handle
    hipMemGenericAllocationHandle_t hc = nullptr;
    void* vc = nullptr;
    rec("c_import", import_fd(rt, &hc, fds[3]));
    (void)H(hipMemAddressReserve)(&vc, kGran, 0, nullptr, 0);
    rec("c_map", H(hipMemMap)(vc, kGran, 0, hc, 0));
    rec("c_access", H(hipMemSetAccess)(vc, kGran, &d, 1));
    rec("c_unmap", H(hipMemUnmap)(vc, kGran));
    rec("c_release", H(hipMemRelease)(hc));
    rec("c_c4", count_of(fds[3]));
    rec("c_release_again", H(hipMemRelease)(hc));
    (void)H(hipGetLastError)();
    rec("c_c4_again", count_of(fds[3]));
    (void)H(hipMemAddressFree)(vc, kGran);
    rec("c_c_after_free", count_of(fds[3]));
    rec("c_leaked_freed", free_leaked_imports(fds[3], "c"));
    rec("c_c_after_kfd_free", count_of(fds[3]));
  }
  {  // D: release while mapped, then unmap
    hipMemGenericAllocationHandle_t hd = nullptr;
    void* vd = nullptr;
    rec("d_import", import_fd(rt, &hd, fds[4]));
    (void)H(hipMemAddressReserve)(&vd, kGran, 0, nullptr, 0);
    rec("d_map", H(hipMemMap)(vd, kGran, 0, hd, 0));
    rec("d_access", H(hipMemSetAccess)(vd, kGran, &d, 1));
    rec("d_release", H(hipMemRelease)(hd));
    rec("d_c_released_mapped", count_of(fds[4]));
    rec("d_unmap", H(hipMemUnmap)(vd, kGran));
    rec("d_c4", count_of(fds[4]));
    (void)H(hipMemAddressFree)(vd, kGran);
    rec("d_c_after_free", count_of(fds[4]));
  }
  std::vector<int> rfds = render_fds();
  rec("render_fds", long(rfds.size()));
  int closed = 0, found = 0;
  for (int r : rfds) {
    drm_prime_handle_ ph{0, 0, fd};
    if (ioctl(r, kPrimeFdToHandle, &ph) == 0) {
      ++found;
      rec("gem_handle", long(ph.handle));
      rec("c_after_lookup", count_of(fd));
      drm_gem_close_ gc{ph.handle, 0};
      if (ioctl(r, kGemClose, &gc) == 0) ++closed;
      drm_gem_close_ gc2{ph.handle, 0};
      rec("second_close_rc", ioctl(r, kGemClose, &gc2));
    }
  }
  rec("prime_lookups", found);
  {
    int imports = 0, frees = 0, maps = 0, unmaps = 0;
    for (int i = 0; i < g_nk; ++i) {
      imports += g_k[i].nr == 0x1D;
      frees += g_k[i].nr == 0x17;
      maps += g_k[i].nr == 0x18;
      unmaps += g_k[i].nr == 0x19;
    }
    rec("kfd_imports", imports);
    rec("kfd_frees", frees);
    rec("kfd_maps", maps);
    rec("kfd_unmaps", unmaps);
  }
  rec("gem_closed", closed);
  rec("c6", count_of(fd));
  (void)H(hipMemAddressFree)(va, kGran);
  if (write(sp[0], "x", 1) != 1) rec("tell_exporter", -1);
  int st = 0;
  waitpid(child, &st, 0);
  rec("exporter_status", st);
  rec("c7_exporter_gone", count_of(fd));
  for (int i = 0; i < kFds; ++i) close(fds[i]);
  out += "}";
  return out.c_str();
}

#ifdef PROBE_MAIN
int main(int argc, char** argv) {
  std::puts(dmabuf_ref_probe(argc > 1 ? std::atoi(argv[1]) : 0));
  return 0;
}
#endif
