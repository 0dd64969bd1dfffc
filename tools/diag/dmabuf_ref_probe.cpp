// Who keeps a broker granule's dma-buf referenced after a tenant released it?
//
// The HBM broker lends a granule again only when no reference to its dma-buf is left outside the
// broker (fdinfo "count"). Measured in round 4-5: a tenant's references stay until its process is
// torn down, even after hipMemUnmap + hipMemRelease of the imported handle, so a replacement pod
// waits for the retired pod's process teardown (~70-110 ms). This probe follows the count through
// one import: a child process exports a 1 GiB handle and sends the fd (SCM_RIGHTS), as the broker
// does, and stays alive; this process imports it, as a tenant does:
//
//   c0  exported fd only
//   c1  after hipMemImportFromShareableHandle
//   c2  after hipMemMap + hipMemSetAccess
//   c3  after hipMemUnmap
//   c4  after hipMemRelease of the imported handle
//   c5  after hipDeviceSynchronize
//   then, on every render-node fd of this process, DRM_IOCTL_PRIME_FD_TO_HANDLE of the dma-buf
//   (the GEM handle this DRM file holds for it, if any) and DRM_IOCTL_GEM_CLOSE of that handle:
//   c6  after those closes
//
//   g++ -std=c++17 -O1 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o tools/diag/build/dmabuf_ref_probe \
//       tools/diag/dmabuf_ref_probe.cpp -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
#include <hip/hip_runtime.h>

#include <dirent.h>
#include <fcntl.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <time.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {
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
}  // namespace

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

int main() {
  const size_t gran = 1ull << 30;
  hipMemAllocationProp p;
  std::memset(&p, 0, sizeof p);
  p.type = hipMemAllocationTypePinned;
  p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
  p.location.type = hipMemLocationTypeDevice;
  p.location.id = 0;
  int sp[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sp)) return 2;
  pid_t child = fork();  // before any HIP call in either process
  if (child == 0) {      // the exporter (the broker's part)
    close(sp[0]);
    hipMemGenericAllocationHandle_t h = nullptr, h2 = nullptr;
    int efd = -1, efd2 = -1;
    if (hipSetDevice(0) != hipSuccess || hipMemCreate(&h, gran, &p, 0) != hipSuccess ||
        hipMemExportToShareableHandle(&efd, h, hipMemHandleTypePosixFileDescriptor, 0) != hipSuccess ||
        hipMemCreate(&h2, gran, &p, 0) != hipSuccess ||
        hipMemExportToShareableHandle(&efd2, h2, hipMemHandleTypePosixFileDescriptor, 0) != hipSuccess)
      _exit(3);
    send_fd(sp[1], efd);
    send_fd(sp[1], efd2);
    char b;
    if (read(sp[1], &b, 1) < 0) _exit(4);  // until the tenant is done
    _exit(0);
  }
  close(sp[1]);
  int fd = recv_fd(sp[0]);
  int fd2 = recv_fd(sp[0]);
  if (fd < 0 || fd2 < 0) return 3;
  if (hipSetDevice(0) != hipSuccess) return 2;
  int rt = 0;
  (void)hipRuntimeGetVersion(&rt);
  hipMemGenericAllocationHandle_t hi = nullptr;
  std::string o = "{\"runtime_version\": " + std::to_string(rt);
  auto rec = [&](const char* k, long v) { o += std::string(", \"") + k + "\": " + std::to_string(v); };
  rec("c0", count_of(fd));
  hipError_t e = rt < 70100000 ? hipMemImportFromShareableHandle(&hi, &fd, hipMemHandleTypePosixFileDescriptor)
                               : hipMemImportFromShareableHandle(&hi, reinterpret_cast<void*>(static_cast<intptr_t>(fd)),
                                                                 hipMemHandleTypePosixFileDescriptor);
  rec("import", e);
  rec("c1", count_of(fd));
  rec("c_fd2_before", count_of(fd2));
  void* va = nullptr;
  rec("reserve", hipMemAddressReserve(&va, gran, 0, nullptr, 0));
  auto now_us = [] {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return long(t.tv_sec) * 1000000 + t.tv_nsec / 1000;
  };
  long t0 = now_us();
  rec("map", hipMemMap(va, gran, 0, hi, 0));
  rec("first_map_us", now_us() - t0);
  hipMemAccessDesc d;
  std::memset(&d, 0, sizeof d);
  d.location.type = hipMemLocationTypeDevice;
  d.location.id = 0;
  d.flags = hipMemAccessFlagsProtReadWrite;
  rec("access", hipMemSetAccess(va, gran, &d, 1));
  rec("memset", hipMemset(va, 0, 4096));
  rec("sync0", hipDeviceSynchronize());
  rec("c2", count_of(fd));
  rec("unmap", hipMemUnmap(va, gran));
  rec("c3", count_of(fd));
  rec("release_imported", hipMemRelease(hi));
  rec("c4", count_of(fd));
  rec("sync", hipDeviceSynchronize());
  rec("c5", count_of(fd));
  {
    // left alone, does the count come down while the process lives?
    int c = count_of(fd), ms = 0;
    while (ms < 300 && count_of(fd) == c) {
      usleep(1000);
      ++ms;
    }
    rec("c5_after_wait", count_of(fd));
    rec("c5_wait_ms", ms);
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
      // a second close of the same handle: if the lookup created a handle of its own, the first
      // close removed it; if the import had one, it is gone as well now
      drm_gem_close_ gc2{ph.handle, 0};
      rec("second_close_rc", ioctl(r, kGemClose, &gc2));
    }
  }
  rec("prime_lookups", found);
  rec("gem_closed", closed);
  rec("c6", count_of(fd));
  {
    // a second granule into a fresh range: is the first map's cost once per process?
    hipMemGenericAllocationHandle_t h2 = nullptr;
    void* va2 = nullptr;
    long a = now_us();
    hipError_t ie = rt < 70100000 ? hipMemImportFromShareableHandle(&h2, &fd2, hipMemHandleTypePosixFileDescriptor)
                                  : hipMemImportFromShareableHandle(
                                        &h2, reinterpret_cast<void*>(static_cast<intptr_t>(fd2)),
                                        hipMemHandleTypePosixFileDescriptor);
    long b = now_us();
    rec("second_import", ie);
    rec("second_import_us", b - a);
    (void)hipMemAddressReserve(&va2, gran, 0, nullptr, 0);
    long c = now_us();
    rec("second_map", hipMemMap(va2, gran, 0, h2, 0));
    rec("second_map_us", now_us() - c);
    long e2 = now_us();
    rec("second_access", hipMemSetAccess(va2, gran, &d, 1));
    rec("second_access_us", now_us() - e2);
    (void)hipMemUnmap(va2, gran);
    (void)hipMemRelease(h2);
    (void)hipMemAddressFree(va2, gran);
    rec("c_second_released", count_of(fd2));
  }
  (void)hipMemAddressFree(va, gran);
  if (write(sp[0], "x", 1) != 1) rec("tell_exporter", -1);
  int st = 0;
  waitpid(child, &st, 0);
  rec("exporter_status", st);
  rec("c7_exporter_gone", count_of(fd));
  close(fd);
  std::puts((o + "}").c_str());
  return 0;
}
