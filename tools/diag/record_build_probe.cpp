#include <fcntl.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>
#include <cstdio>
#include <cstring>
#include <string>
#include <cstdint>
static int64_t ns() { timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec; }
const char* kB64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
void b64_append(std::string* out, const uint8_t* p, size_t n) {
  size_t i = 0;
  for (; i + 3 <= n; i += 3) { uint32_t v = (uint32_t)p[i] << 16 | (uint32_t)p[i + 1] << 8 | p[i + 2];
    out->push_back(kB64[v >> 18]); out->push_back(kB64[v >> 12 & 63]); out->push_back(kB64[v >> 6 & 63]); out->push_back(kB64[v & 63]); }
}
int main(int argc, char** argv) {
  size_t size = 32 << 20;
  int fd = open(argv[1], O_RDWR | O_CREAT | O_TRUNC, 0600);
  if (ftruncate(fd, size)) return 1; posix_fallocate(fd, 0, size);
  uint8_t* p = (uint8_t*)mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  volatile uint8_t* vp = p; for (size_t o = 0; o < size; o += 4096) vp[o] = vp[o];
  std::string head(380, 'h'), req(24, 'r'); size_t off = 0;
  for (int i = 0; i < 12; i++) {
    if (argc > 2) usleep(atoi(argv[2]));
    int64_t a = ns();
    std::string rec = head; char tb[48]; snprintf(tb, sizeof tb, "%.6f", 1760000000.123456); rec += tb;
    rec += ",\"req\":\""; b64_append(&rec, (const uint8_t*)req.data(), req.size()); rec += "\"}\n";
    int64_t b = ns();
    memcpy(p + off, rec.data(), rec.size()); off += rec.size();
    int64_t c = ns();
    printf("%d build %.1f us copy %.1f us\n", i, (b - a) / 1e3, (c - b) / 1e3);
  }
}
