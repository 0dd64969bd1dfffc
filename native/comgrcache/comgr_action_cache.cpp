// libgpushare_comgrcache.so: a whole-pipeline cache in front of comgr for the HIP runtime's own
// compiles, preloaded into shared pods next to the quota shim.
//
// At a process's first stream the HIP runtime builds its blit (copy / fill) kernels from OpenCL
// source through comgr: precompiled headers, source -> bitcode with the device libraries, link,
// codegen, link to an executable. comgr's own cache (AMD_COMGR_CACHE) covers only the codegen
// step, so a pod still spends ~78 ms of its start in the rest (profiles/r6/first_stream/). This
// library caches every step of that pipeline by the full content of its inputs:
//
//  * the runtime loads comgr with dlopen and takes each entry point with dlsym. The library
//    defines dlsym: a lookup of "amd_comgr_do_action" in a comgr handle returns gs_do_action
//    (which calls the real one on a miss); every other lookup is a guaranteed tail call into
//    the C library's dlsym (comgr_dlsym.c), so RTLD_NEXT still resolves relative to the real caller;
//  * the key is a 128-bit hash of the comgr build (version, library size and mtime), the action
//    kind, ISA, language, options and every input object's kind, name and bytes. (Not the
//    working directory: comgr 3.0 faults reading an unset one. The cached steps take their
//    inputs as data objects, not files, so it only matters to a relative -I in the options.) A hit rebuilds the result set from the entry; anything unexpected (a non-empty result
//    set, a short or corrupt entry, a comgr debugging variable) runs the real action;
//  * entries are written only by a fill (GPUSHARE_COMGR_ACTION_CACHE_WRITE=1: the DaemonSet's
//    init container, quota/comgr_cache.py), atomically (temporary file + rename). Pods get the
//    directory read-only and never write, so no pod can place code in another pod's runtime.
//
// Env: GPUSHARE_COMGR_ACTION_CACHE=<dir> enables it; GPUSHARE_COMGR_ACTION_CACHE_LOG=1 prints one
// line per cached action to stderr. Host code only; the interposer is built with clang for its
// guaranteed tail call (__attribute__((musttail))).
#include <amd_comgr/amd_comgr.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#define GS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

using dlsym_fn = void* (*)(void*, const char*);
dlsym_fn g_real_dlsym = nullptr;

// (not instrumented in a sanitizer build: a sanitizer runtime resolves its interceptors with dlsym
// before its shadow memory exists)
#define GS_NO_SANITIZE __attribute__((no_sanitize("address", "undefined", "thread")))

GS_NO_SANITIZE void resolve_real_dlsym() {
  void* p = dlvsym(RTLD_NEXT, "dlsym", "GLIBC_2.34");
  if (p == nullptr) p = dlvsym(RTLD_NEXT, "dlsym", "GLIBC_2.2.5");
  if (p == nullptr) {
    static const char msg[] = "gpushare-comgr: the C library's dlsym was not found\n";
    ssize_t r = write(2, msg, sizeof msg - 1);
    (void)r;
    abort();
  }
  __atomic_store_n(&g_real_dlsym, reinterpret_cast<dlsym_fn>(p), __ATOMIC_RELEASE);
}

struct Comgr {
  decltype(&amd_comgr_do_action) do_action = nullptr;
  decltype(&amd_comgr_get_version) get_version = nullptr;
  decltype(&amd_comgr_action_data_count) data_count = nullptr;
  decltype(&amd_comgr_action_data_get_data) get_item = nullptr;
  decltype(&amd_comgr_get_data) get_data = nullptr;
  decltype(&amd_comgr_get_data_name) get_name = nullptr;
  decltype(&amd_comgr_release_data) release = nullptr;
  decltype(&amd_comgr_create_data) create = nullptr;
  decltype(&amd_comgr_set_data) set_data = nullptr;
  decltype(&amd_comgr_set_data_name) set_name = nullptr;
  decltype(&amd_comgr_data_set_add) set_add = nullptr;
  decltype(&amd_comgr_data_set_remove) set_remove = nullptr;
  decltype(&amd_comgr_action_info_get_isa_name) info_isa = nullptr;
  decltype(&amd_comgr_action_info_get_language) info_lang = nullptr;
  decltype(&amd_comgr_action_info_get_option_list_count) info_nopt = nullptr;
  decltype(&amd_comgr_action_info_get_option_list_item) info_opt = nullptr;
  uint64_t build[4] = {0, 0, 0, 0};   // version major, minor; library size, mtime
};

Comgr g_c;
std::mutex g_mu;
bool g_bound = false;
std::string g_dir;
bool g_write = false, g_log = false, g_on = false;
std::once_flag g_env_once;
std::atomic<uint64_t> g_stat[5];   // hits, misses, stores, bypassed, errors

void read_env() {
  const char* d = getenv("GPUSHARE_COMGR_ACTION_CACHE");
  if (d == nullptr || *d == '\0') return;
  g_dir = d;
  const char* w = getenv("GPUSHARE_COMGR_ACTION_CACHE_WRITE");
  g_write = w != nullptr && std::strcmp(w, "1") == 0;
  const char* l = getenv("GPUSHARE_COMGR_ACTION_CACHE_LOG");
  g_log = l != nullptr && std::strcmp(l, "1") == 0;
  // comgr's own debugging output (temporaries, verbose logs) is not in the key: run it for real
  g_on = getenv("AMD_COMGR_SAVE_TEMPS") == nullptr && getenv("AMD_COMGR_EMIT_VERBOSE_LOGS") == nullptr;
}

bool enabled() {
  std::call_once(g_env_once, read_env);
  return g_on;
}

// the pipeline steps of a runtime's own compile: each a pure function of the key's inputs
bool cacheable(amd_comgr_action_kind_t k) {
  return k == AMD_COMGR_ACTION_COMPILE_SOURCE_WITH_DEVICE_LIBS_TO_BC || k == AMD_COMGR_ACTION_LINK_BC_TO_BC ||
         k == AMD_COMGR_ACTION_CODEGEN_BC_TO_RELOCATABLE || k == AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE;
}

// Two independent 64-bit lanes over 8-byte words, finalised with murmur3's fmix64: not a
// cryptographic hash (entries come only from the trusted fill), a key with no practical
// collisions between different compiles.
struct Hash {
  uint64_t a = 0x243f6a8885a308d3ull, b = 0x13198a2e03707344ull, n = 0;
  static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
  void word(uint64_t w) {
    a = (a ^ w) * 0x9e3779b97f4a7c15ull;
    a ^= a >> 29;
    b = rotl(b + w, 31) * 0xc2b2ae3d27d4eb4full;
  }
  void bytes(const void* p, size_t len) {
    const unsigned char* s = static_cast<const unsigned char*>(p);
    word(len ^ 0xa0761d6478bd642full);
    size_t i = 0;
    for (; i + 32 <= len; i += 32) {          // four words per trip: the PCH input is megabytes
      uint64_t w[4];
      std::memcpy(w, s + i, 32);
      word(w[0]);
      word(w[1]);
      word(w[2]);
      word(w[3]);
    }
    for (; i + 8 <= len; i += 8) {
      uint64_t w;
      std::memcpy(&w, s + i, 8);
      word(w);
    }
    if (i < len) {
      uint64_t w = 0;
      std::memcpy(&w, s + i, len - i);
      word(w ^ (uint64_t(len - i) << 56));
    }
    n += len;
  }
  void u64(uint64_t v) { bytes(&v, sizeof v); }
  void str(const std::string& s) { bytes(s.data(), s.size()); }
  static uint64_t fmix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
  }
  std::string hex() const {
    char out[33];
    std::snprintf(out, sizeof out, "%016llx%016llx", (unsigned long long)fmix(a ^ n),
                  (unsigned long long)fmix(b + rotl(a, 17)));
    return out;
  }
  uint64_t sum() const { return fmix(a ^ rotl(b, 23) ^ n); }
};

// a size-query-then-read string getter of comgr (sizes include the terminating NUL)
template <class F>
bool get_string(F f, std::string* out) {
  size_t n = 0;
  if (f(&n, nullptr) != AMD_COMGR_STATUS_SUCCESS) return false;
  out->assign(n, '\0');
  if (n && f(&n, &(*out)[0]) != AMD_COMGR_STATUS_SUCCESS) return false;
  while (!out->empty() && out->back() == '\0') out->pop_back();
  return true;
}

bool data_bytes(amd_comgr_data_t d, std::string* name, std::string* bytes) {
  if (!get_string([&](size_t* n, char* p) { return g_c.get_name(d, n, p); }, name)) return false;
  size_t n = 0;
  if (g_c.get_data(d, &n, nullptr) != AMD_COMGR_STATUS_SUCCESS) return false;
  bytes->resize(n);
  return n == 0 || g_c.get_data(d, &n, &(*bytes)[0]) == AMD_COMGR_STATUS_SUCCESS;
}

struct Obj {
  uint32_t kind;
  std::string name, bytes;
};

// every object of a data set, kind by kind (kinds comgr does not know are skipped)
bool set_objects(amd_comgr_data_set_t s, std::vector<Obj>* out) {
  for (uint32_t k = AMD_COMGR_DATA_KIND_SOURCE; k <= AMD_COMGR_DATA_KIND_LAST; ++k) {
    size_t n = 0;
    if (g_c.data_count(s, amd_comgr_data_kind_t(k), &n) != AMD_COMGR_STATUS_SUCCESS) continue;
    for (size_t i = 0; i < n; ++i) {
      amd_comgr_data_t d;
      if (g_c.get_item(s, amd_comgr_data_kind_t(k), i, &d) != AMD_COMGR_STATUS_SUCCESS) return false;
      Obj o{k, {}, {}};
      bool ok = data_bytes(d, &o.name, &o.bytes);
      g_c.release(d);
      if (!ok) return false;
      out->push_back(std::move(o));
    }
  }
  return true;
}

bool set_empty(amd_comgr_data_set_t s) {
  for (uint32_t k = AMD_COMGR_DATA_KIND_SOURCE; k <= AMD_COMGR_DATA_KIND_LAST; ++k) {
    size_t n = 0;
    if (g_c.data_count(s, amd_comgr_data_kind_t(k), &n) == AMD_COMGR_STATUS_SUCCESS && n) return false;
  }
  return true;
}

bool make_key(amd_comgr_action_kind_t kind, amd_comgr_action_info_t info, amd_comgr_data_set_t in,
              std::string* key) {
  Hash h;
  h.str("gpushare-comgr-action-1");
  for (uint64_t v : g_c.build) h.u64(v);
  h.u64(uint64_t(kind));
  std::string s;
  if (!get_string([&](size_t* n, char* p) { return g_c.info_isa(info, n, p); }, &s)) return false;
  h.str(s);
  amd_comgr_language_t lang;
  if (g_c.info_lang(info, &lang) != AMD_COMGR_STATUS_SUCCESS) return false;
  h.u64(uint64_t(lang));
  size_t nopt = 0;
  if (g_c.info_nopt(info, &nopt) != AMD_COMGR_STATUS_SUCCESS) return false;
  h.u64(nopt);
  for (size_t i = 0; i < nopt; ++i) {
    if (!get_string([&](size_t* n, char* p) { return g_c.info_opt(info, i, n, p); }, &s)) return false;
    h.str(s);
  }
  std::vector<Obj> objs;
  if (!set_objects(in, &objs)) return false;
  for (const Obj& o : objs) {
    // a log or diagnostic passed along from the previous step is not an input comgr compiles
    // (and a cached step leaves an empty one out)
    if (o.kind == AMD_COMGR_DATA_KIND_LOG || o.kind == AMD_COMGR_DATA_KIND_DIAGNOSTIC) continue;
    h.u64(o.kind);
    h.str(o.name);
    h.str(o.bytes);
  }
  *key = h.hex();
  return true;
}

// entry: "GSCA0001" | u32 count | count x (u32 kind, u32 name_len, u64 size, name, bytes) | u64 sum
const char kMagic[8] = {'G', 'S', 'C', 'A', '0', '0', '0', '1'};

bool read_file(const std::string& path, std::string* out) {
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  struct stat st;
  bool ok = fstat(fd, &st) == 0 && st.st_size > 0 && st.st_size < (1ll << 31);
  if (ok) {
    out->resize(size_t(st.st_size));
    size_t got = 0;
    while (got < out->size()) {
      ssize_t r = read(fd, &(*out)[got], out->size() - got);
      if (r <= 0) break;
      got += size_t(r);
    }
    ok = got == out->size();
  }
  close(fd);
  return ok;
}

bool parse(const std::string& f, std::vector<Obj>* objs) {
  if (f.size() < sizeof kMagic + 4 + 8 || std::memcmp(f.data(), kMagic, sizeof kMagic) != 0) return false;
  Hash h;
  h.bytes(f.data(), f.size() - 8);
  uint64_t sum;
  std::memcpy(&sum, f.data() + f.size() - 8, 8);
  if (sum != h.sum()) return false;
  size_t at = sizeof kMagic, end = f.size() - 8;
  uint32_t count;
  std::memcpy(&count, f.data() + at, 4);
  at += 4;
  for (uint32_t i = 0; i < count; ++i) {
    if (end - at < 16) return false;
    uint32_t kind, nlen;
    uint64_t size;
    std::memcpy(&kind, f.data() + at, 4);
    std::memcpy(&nlen, f.data() + at + 4, 4);
    std::memcpy(&size, f.data() + at + 8, 8);
    at += 16;
    if (kind < AMD_COMGR_DATA_KIND_SOURCE || kind > AMD_COMGR_DATA_KIND_LAST || nlen > end - at ||
        size > end - at - nlen)
      return false;
    objs->push_back(Obj{kind, f.substr(at, nlen), f.substr(at + nlen, size)});
    at += nlen + size;
  }
  return at == end;
}

bool load(const std::string& path, amd_comgr_data_set_t out) {
  std::string f;
  std::vector<Obj> objs;
  if (!read_file(path, &f) || !parse(f, &objs)) return false;
  std::vector<uint32_t> added;
  for (const Obj& o : objs) {
    // an empty log or diagnostic (a quiet step) is left out: comgr refuses to set 0 bytes, and an
    // object created empty cannot be read back (the next step's key). Readers count them first.
    if (o.bytes.empty() && (o.kind == AMD_COMGR_DATA_KIND_LOG || o.kind == AMD_COMGR_DATA_KIND_DIAGNOSTIC)) continue;
    amd_comgr_data_t d;
    if (g_c.create(amd_comgr_data_kind_t(o.kind), &d) != AMD_COMGR_STATUS_SUCCESS) goto undo;
    {
      bool ok = g_c.set_data(d, o.bytes.size(), o.bytes.data()) == AMD_COMGR_STATUS_SUCCESS &&
                (o.name.empty() || g_c.set_name(d, o.name.c_str()) == AMD_COMGR_STATUS_SUCCESS) &&
                g_c.set_add(out, d) == AMD_COMGR_STATUS_SUCCESS;
      g_c.release(d);                       // the set holds its own reference
      if (!ok) goto undo;
    }
    added.push_back(o.kind);
  }
  return true;
undo:
  for (uint32_t k : added) g_c.set_remove(out, amd_comgr_data_kind_t(k));
  g_stat[4].fetch_add(1, std::memory_order_relaxed);
  return false;
}

void store(const std::string& path, amd_comgr_data_set_t out) {
  std::vector<Obj> objs;
  if (!set_objects(out, &objs)) return;
  std::string f(kMagic, sizeof kMagic);
  uint32_t count = uint32_t(objs.size());
  f.append(reinterpret_cast<const char*>(&count), 4);
  for (const Obj& o : objs) {
    uint32_t nlen = uint32_t(o.name.size());
    uint64_t size = o.bytes.size();
    f.append(reinterpret_cast<const char*>(&o.kind), 4);
    f.append(reinterpret_cast<const char*>(&nlen), 4);
    f.append(reinterpret_cast<const char*>(&size), 8);
    f += o.name;
    f += o.bytes;
  }
  Hash h;
  h.bytes(f.data(), f.size());
  uint64_t sum = h.sum();
  f.append(reinterpret_cast<const char*>(&sum), 8);
  std::string tmp = g_dir + "/.gsa-tmp-" + std::to_string(getpid()) + "-" +
                    std::to_string(std::chrono::steady_clock::now().time_since_epoch().count());
  int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
  if (fd < 0) return;
  size_t put = 0;
  while (put < f.size()) {
    ssize_t w = write(fd, f.data() + put, f.size() - put);
    if (w <= 0) break;
    put += size_t(w);
  }
  bool ok = put == f.size();
  ok = close(fd) == 0 && ok;
  if (ok && rename(tmp.c_str(), path.c_str()) == 0) {
    g_stat[2].fetch_add(1, std::memory_order_relaxed);
  } else {
    unlink(tmp.c_str());
    g_stat[4].fetch_add(1, std::memory_order_relaxed);
  }
}

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

amd_comgr_status_t gs_do_action(amd_comgr_action_kind_t kind, amd_comgr_action_info_t info,
                                amd_comgr_data_set_t in, amd_comgr_data_set_t out) {
  if (!cacheable(kind)) return g_c.do_action(kind, info, in, out);
  auto t0 = std::chrono::steady_clock::now();
  std::string key;
  if (!set_empty(out) || !make_key(kind, info, in, &key)) {
    g_stat[3].fetch_add(1, std::memory_order_relaxed);
    return g_c.do_action(kind, info, in, out);
  }
  std::string path = g_dir + "/gsa-" + key;
  if (load(path, out)) {
    g_stat[0].fetch_add(1, std::memory_order_relaxed);
    if (g_log) std::fprintf(stderr, "gpushare-comgr: action %d hit %s %.3f ms\n", int(kind), key.c_str(), ms_since(t0));
    return AMD_COMGR_STATUS_SUCCESS;
  }
  amd_comgr_status_t st = g_c.do_action(kind, info, in, out);
  g_stat[1].fetch_add(1, std::memory_order_relaxed);
  if (st == AMD_COMGR_STATUS_SUCCESS && g_write) store(path, out);
  if (g_log) std::fprintf(stderr, "gpushare-comgr: action %d miss %s %.3f ms\n", int(kind), key.c_str(), ms_since(t0));
  return st;
}

template <class T>
bool bind_one(void* h, const char* name, T* slot) {
  *slot = reinterpret_cast<T>(g_real_dlsym(h, name));
  return *slot != nullptr;
}

// the runtime asked a comgr handle for amd_comgr_do_action: bind the wrapper to that comgr
void* wrap(void* handle) {
  if (!enabled()) return nullptr;
  if (__atomic_load_n(&g_real_dlsym, __ATOMIC_ACQUIRE) == nullptr) resolve_real_dlsym();
  void* real = g_real_dlsym(handle, "amd_comgr_do_action");
  if (real == nullptr) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_bound) return reinterpret_cast<void*>(g_c.do_action) == real ? reinterpret_cast<void*>(&gs_do_action) : real;
  Comgr c;
  bool ok = bind_one(handle, "amd_comgr_do_action", &c.do_action) && bind_one(handle, "amd_comgr_get_version", &c.get_version) &&
            bind_one(handle, "amd_comgr_action_data_count", &c.data_count) &&
            bind_one(handle, "amd_comgr_action_data_get_data", &c.get_item) &&
            bind_one(handle, "amd_comgr_get_data", &c.get_data) && bind_one(handle, "amd_comgr_get_data_name", &c.get_name) &&
            bind_one(handle, "amd_comgr_release_data", &c.release) && bind_one(handle, "amd_comgr_create_data", &c.create) &&
            bind_one(handle, "amd_comgr_set_data", &c.set_data) && bind_one(handle, "amd_comgr_set_data_name", &c.set_name) &&
            bind_one(handle, "amd_comgr_data_set_add", &c.set_add) && bind_one(handle, "amd_comgr_data_set_remove", &c.set_remove) &&
            bind_one(handle, "amd_comgr_action_info_get_isa_name", &c.info_isa) &&
            bind_one(handle, "amd_comgr_action_info_get_language", &c.info_lang) &&
            bind_one(handle, "amd_comgr_action_info_get_option_list_count", &c.info_nopt) &&
            bind_one(handle, "amd_comgr_action_info_get_option_list_item", &c.info_opt);
  if (!ok) return real;
  size_t major = 0, minor = 0;
  c.get_version(&major, &minor);
  c.build[0] = major;
  c.build[1] = minor;
  Dl_info dl;
  struct stat st;
  if (dladdr(real, &dl) == 0 || dl.dli_fname == nullptr || stat(dl.dli_fname, &st) != 0) return real;
  c.build[2] = uint64_t(st.st_size);
  c.build[3] = uint64_t(st.st_mtim.tv_sec) * 1000000000ull + uint64_t(st.st_mtim.tv_nsec);
  g_c = c;
  g_bound = true;
  return reinterpret_cast<void*>(&gs_do_action);
}

}  // namespace

// the dlsym interposer (comgr_dlsym.c, C: glibc declares dlsym noexcept in C++, and a tail call
// cannot leave a noexcept frame) calls these two
extern "C" __attribute__((visibility("hidden"))) void* gs_comgr_wrap(void* handle) { return wrap(handle); }

extern "C" __attribute__((visibility("hidden"))) GS_NO_SANITIZE dlsym_fn gs_comgr_real_dlsym() {
  dlsym_fn f = __atomic_load_n(&g_real_dlsym, __ATOMIC_ACQUIRE);
  if (__builtin_expect(f == nullptr, 0)) {
    resolve_real_dlsym();
    f = __atomic_load_n(&g_real_dlsym, __ATOMIC_ACQUIRE);
  }
  return f;
}

// hits, misses, stores, bypassed, errors (tests and the fill's report)
GS_EXPORT int gpushare_comgr_cache_stats(uint64_t* out, int n) {
  int k = n < 5 ? n : 5;
  for (int i = 0; i < k; ++i) out[i] = g_stat[i].load(std::memory_order_relaxed);
  return k;
}
