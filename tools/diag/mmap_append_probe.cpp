#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <cstdio>
#include <cstring>
#include <string>
#include <cstdint>
static int64_t ns() { timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec; }
int main(int argc, char** argv) {
  const char* path = argv[1]; size_t size = 32 << 20; int gap_ms = atoi(argv[2]);
  int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0600);
  ftruncate(fd, size); posix_fallocate(fd, 0, size);
  uint8_t* p = (uint8_t*)mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  volatile uint8_t* vp = p; for (size_t o = 0; o < size; o += 4096) vp[o] = vp[o];
  std::string rec(1000, 'x'); size_t off = 0;
  for (int i = 0; i < atoi(argv[3]); i++) {
    usleep(gap_ms * 1000);
    int64_t a = ns(); memcpy(p + off, rec.data(), rec.size()); int64_t b = ns();
    printf("%d off=%zu page=%zu %.1f us\n", i, off, off / 4096, (b - a) / 1e3);
    off += rec.size();
  }
}
