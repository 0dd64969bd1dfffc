// VMM from the broker arena: PyTorch's expandable segments and any other program that
// reserves address space and maps physical handles into it (shim.h lists the units and the lock
// order).
#include "shim.h"

#include <stdlib.h>
#include <string.h>

namespace gs {
namespace {
// ---- VMM from the arena (PyTorch's expandable segments) ----------------------------------------
// A VMM user reserves a large VA range (hipMemAddressReserve), creates small physical handles
// (hipMemCreate, 2 / 20 MiB pages for PyTorch) and maps them one after another into the range.
// Physical handles of the arena cannot be cut into pages, so the shim lends whole granules:
// a reservation of >= 1 GiB (a "window") is aligned to the granule, its granule-sized slots are
// backed on demand by arena granules (unmapped from the arena's own range and mapped into the
// slot), and the user's handles are stand-ins whose map is a no-op inside a backed slot. A slot
// whose pages are all unmapped gives its granule back to the arena. When no granule is free, the
// slot is served by real handles from the driver (charged to the quota as before).
constexpr int kMaxWin = 64;
constexpr uint64_t kVHandleMagic = 0x67737668616e646cull;  // "gsvhandl"

struct Win {
  char* base;
  uint64_t size;
  char* vbase;     // the reservation it lies in (larger when the runtime ignored the alignment)
  uint64_t vsize;
  int nslots;
  int32_t* slot_g;      // arena granule backing the slot, -1 none
  uint64_t* slot_used;  // bytes of stand-in pages mapped in the slot (arena-backed slots)
  uint32_t* slot_real;  // real (driver) pieces mapped in the slot
};
Win g_win[kMaxWin];
int g_nwin = 0;

struct VPiece {
  char* va;
  uint64_t len;
  hipMemGenericAllocationHandle_t h;  // real handle (driver), or nullptr: inside an arena slot
};
struct VHandle {
  uint64_t magic;
  uint64_t size;
  hipMemAllocationProp prop;
  unsigned long long flags;
  char* at;  // mapped at (nullptr: not mapped)
  int retains;  // hipMemRetainAllocationHandle references: each hipMemRelease drops one first
  int npieces;
  VPiece* pieces;
};

// stand-in handles and their mapped addresses: open addressing on the pointer / VA
constexpr uint64_t kVCap = 1 << 17;
uintptr_t* g_vh = nullptr;   // VHandle* set
uintptr_t* g_vva = nullptr;  // VA -> VHandle* (pairs)
uint64_t g_vh_n = 0, g_vva_n = 0, g_pending_bytes = 0;
uint64_t g_vmm_arena_maps = 0, g_vmm_real_pieces = 0, g_vmm_creates = 0, g_slots_backed = 0, g_vmm_span_access = 0;

bool vtables() {
  if (!g_vh) g_vh = static_cast<uintptr_t*>(calloc(kVCap, sizeof(uintptr_t)));
  if (!g_vva) g_vva = static_cast<uintptr_t*>(calloc(2 * kVCap, sizeof(uintptr_t)));
  return g_vh && g_vva;
}
uint64_t vslot(uintptr_t k) { return (k * 0x9E3779B97F4A7C15ull >> 17) & (kVCap - 1); }
constexpr uintptr_t kTomb = ~uintptr_t(0);

bool vh_put(VHandle* h) {
  if (g_vh_n * 2 >= kVCap) return false;
  uintptr_t k = reinterpret_cast<uintptr_t>(h);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1))
    if (!g_vh[i] || g_vh[i] == kTomb) {
      g_vh[i] = k;
      ++g_vh_n;
      return true;
    }
}
bool vh_has(const void* p) {
  if (!g_vh || !p) return false;
  uintptr_t k = reinterpret_cast<uintptr_t>(p);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1)) {
    if (!g_vh[i]) return false;
    if (g_vh[i] == k) return true;
  }
}
void vh_del(VHandle* h) {
  uintptr_t k = reinterpret_cast<uintptr_t>(h);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1)) {
    if (!g_vh[i]) return;
    if (g_vh[i] == k) {
      g_vh[i] = kTomb;
      --g_vh_n;
      return;
    }
  }
}
bool vva_put(char* va, VHandle* h) {
  if (g_vva_n * 2 >= kVCap) return false;
  uintptr_t k = reinterpret_cast<uintptr_t>(va);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1))
    if (!g_vva[2 * i] || g_vva[2 * i] == kTomb) {
      g_vva[2 * i] = k;
      g_vva[2 * i + 1] = reinterpret_cast<uintptr_t>(h);
      ++g_vva_n;
      return true;
    }
}
VHandle* vva_take(char* va) {
  if (!g_vva) return nullptr;
  uintptr_t k = reinterpret_cast<uintptr_t>(va);
  for (uint64_t i = vslot(k);; i = (i + 1) & (kVCap - 1)) {
    if (!g_vva[2 * i]) return nullptr;
    if (g_vva[2 * i] == k) {
      g_vva[2 * i] = kTomb;
      --g_vva_n;
      return reinterpret_cast<VHandle*>(g_vva[2 * i + 1]);
    }
  }
}

// where the run of mappings that ends at `at` without a hole begins, in window `w`: whole arena
// slots and the driver pieces mapped in the other slots (g_arena.mu held)
struct Span {
  char* va;
  uint64_t len;
};
int span_cmp(const void* x, const void* y) {
  const char* a = static_cast<const Span*>(x)->va;
  const char* b = static_cast<const Span*>(y)->va;
  return a < b ? -1 : a > b;
}
char* mapped_run_start(Win& w, char* at) {
  uint64_t cap = 256, n = 0;
  Span* v = static_cast<Span*>(malloc(cap * sizeof(Span)));
  for (uint64_t i = 0; v && g_vva && i < kVCap; ++i) {
    uintptr_t k = g_vva[2 * i];
    if (!k || k == kTomb) continue;
    VHandle* h = reinterpret_cast<VHandle*>(g_vva[2 * i + 1]);
    for (int j = 0; j < h->npieces; ++j) {
      VPiece& pc = h->pieces[j];
      if (!pc.h || pc.va < w.base || pc.va >= w.base + w.size) continue;
      if (n == cap) {
        Span* g = static_cast<Span*>(realloc(v, 2 * cap * sizeof(Span)));
        if (!g) break;
        v = g;
        cap *= 2;
      }
      v[n++] = {pc.va, pc.len};
    }
  }
  if (v) qsort(v, n, sizeof(Span), span_cmp);
  char* cur = at;
  while (v && cur > w.base) {
    int s = int(uint64_t(cur - 1 - w.base) / kWinAlign);
    char* st = w.base + uint64_t(s) * kWinAlign;
    if (w.slot_g[s] >= 0) {  // an arena slot: one mapping of its whole granule
      if (cur != st + kWinAlign) break;
      cur = st;
      continue;
    }
    uint64_t lo = 0, hi = n;  // the last driver piece starting below cur
    while (lo < hi) {
      uint64_t mid = (lo + hi) / 2;
      if (v[mid].va < cur) lo = mid + 1;
      else hi = mid;
    }
    if (lo == 0 || v[lo - 1].va + v[lo - 1].len != cur) break;
    cur = v[lo - 1].va;
  }
  free(v);
  return cur;
}


Win* win_of(const char* p, uint64_t len) {
  for (int i = 0; i < g_nwin; ++i)
    if (p >= g_win[i].base && p + len <= g_win[i].base + g_win[i].size) return &g_win[i];
  return nullptr;
}

// back slot s of window w with an arena granule (g_arena.mu held); false: none free (or the
// broker's granule is not the slot size: then every page is the driver's)
bool slot_back(Win& w, int s) {
  Arena& a = g_arena;
  uint64_t off;
  if (a.state.load(std::memory_order_relaxed) != 1 || a.gran != kWinAlign) return false;
  while (a.n < a.total && arena_more_locked(0)) {
  }
  bool got = arena_take_granule(&off);
  while (!got && arena_wait_more(a.gran)) got = arena_take_granule(&off);
  if (!got && arena_extend_locked(a.gran)) got = arena_take_granule(&off);   // beyond the grant
  if (!got) return false;
  int gi = int(off / a.gran);
  auto un = real_hipMemUnmap();
  auto map = real_hipMemMap();
  char* slot = w.base + uint64_t(s) * kWinAlign;
  Depth d;
  if (!un || !map || un(a.base + off, a.gran) != hipSuccess) {
    arena_free(off);
    return false;
  }
  if (map(slot, a.gran, 0, a.h[gi], 0) != hipSuccess || !set_rw(slot, a.gran, g_dev)) {
    // back where it was: the arena's own range keeps every granule it does not lend
    if (map(a.base + off, a.gran, 0, a.h[gi], 0) == hipSuccess) set_rw(a.base + off, a.gran, g_dev);
    arena_free(off);
    return false;
  }
  w.slot_g[s] = gi;
  w.slot_used[s] = 0;
  ++g_slots_backed;
  return true;
}

// the slot's last page is gone: its granule goes back to the arena (g_arena.mu held)
void slot_return(Win& w, int s) {
  Arena& a = g_arena;
  int gi = w.slot_g[s];
  if (gi < 0) return;
  auto un = real_hipMemUnmap();
  auto map = real_hipMemMap();
  char* slot = w.base + uint64_t(s) * kWinAlign;
  Depth d;
  if (auto sync = real_hipDeviceSynchronize()) (void)sync();   // nothing may still use it when it moves
  if (un) (void)un(slot, a.gran);
  if (map && map(a.base + uint64_t(gi) * a.gran, a.gran, 0, a.h[gi], 0) == hipSuccess)
    set_rw(a.base + uint64_t(gi) * a.gran, a.gran, g_dev);
  arena_free(uint64_t(gi) * a.gran);
  w.slot_g[s] = -1;
  w.slot_used[s] = 0;
}

// bytes a new stand-in handle could still be given: free arena granules, unmapped room in the
// backed slots, less what stand-ins created but not mapped yet will take (g_arena.mu held)
uint64_t vmm_room() {
  Arena& a = g_arena;
  uint64_t room = a.size - a.used;
  for (int i = 0; i < g_nwin; ++i)
    for (int s = 0; s < g_win[i].nslots; ++s)
      if (g_win[i].slot_g[s] >= 0) room += kWinAlign - g_win[i].slot_used[s];
  return room > g_pending_bytes ? room - g_pending_bytes : 0;
}

hipError_t real_create_charged(hipMemGenericAllocationHandle_t* h, size_t size, const hipMemAllocationProp* prop,
                               unsigned long long flags);

// map stand-in `v` at [va, va + v->size) inside window `w` (g_arena.mu held)
hipError_t vmm_map(Win& w, VHandle* v, char* va) {
  uint64_t lo = uint64_t(va - w.base), hi = lo + v->size;
  int s0 = int(lo / kWinAlign), s1 = int((hi - 1) / kWinAlign);
  v->pieces = static_cast<VPiece*>(calloc(size_t(s1 - s0 + 1), sizeof(VPiece)));
  if (!v->pieces) return hipErrorOutOfMemory;
  v->npieces = 0;
  v->at = va;  // (vmm_unmap undoes a partial map)
  auto map = real_hipMemMap();
  for (int s = s0; s <= s1; ++s) {
    uint64_t plo = s == s0 ? lo : uint64_t(s) * kWinAlign;
    uint64_t phi = s == s1 ? hi : uint64_t(s + 1) * kWinAlign;
    VPiece& pc = v->pieces[v->npieces];
    pc.va = w.base + plo;
    pc.len = phi - plo;
    pc.h = nullptr;
    if (w.slot_g[s] < 0 && w.slot_real[s] == 0) slot_back(w, s);
    if (w.slot_g[s] >= 0) {
      w.slot_used[s] += pc.len;
      ++g_vmm_arena_maps;
    } else {
      // the driver: a real handle of this piece's size, mapped in the slot (charged as any other)
      hipError_t e = real_create_charged(&pc.h, pc.len, &v->prop, v->flags);
      if (e == hipSuccess) {
        Depth d;
        e = map ? map(pc.va, pc.len, 0, pc.h, 0) : hipErrorNotInitialized;
        if (e != hipSuccess) (void)hipMemRelease(pc.h);
      }
      if (e != hipSuccess) {
        logf(1, "vmm: driver piece of %llu bytes at slot %d + %llu: error %d", (unsigned long long)pc.len, s,
             (unsigned long long)(plo - uint64_t(s) * kWinAlign), int(e));
        return e;  // the caller undoes the pieces mapped so far
      }
      ++w.slot_real[s];
      ++g_vmm_real_pieces;
      logf(2, "vmm: driver piece of %llu bytes mapped at +%llu", (unsigned long long)pc.len, (unsigned long long)plo);
    }
    ++v->npieces;
  }
  return hipSuccess;
}

// unmap stand-in `v` (g_arena.mu held); its real pieces are released with it (hipMemRelease)
void vmm_unmap(VHandle* v) {
  Win* w = v->at ? win_of(v->at, v->size) : nullptr;
  auto un = real_hipMemUnmap();
  for (int i = 0; i < v->npieces && w; ++i) {
    VPiece& pc = v->pieces[i];
    int s = int(uint64_t(pc.va - w->base) / kWinAlign);
    if (pc.h) {
      Depth d;
      if (un) (void)un(pc.va, pc.len);
      --w->slot_real[s];
    } else if (w->slot_g[s] >= 0) {
      w->slot_used[s] -= pc.len;
      if (w->slot_used[s] == 0) slot_return(*w, s);
    }
  }
  v->at = nullptr;
}

void vmm_release_pieces(VHandle* v) {
  for (int i = 0; i < v->npieces; ++i)
    if (v->pieces[i].h) (void)hipMemRelease(v->pieces[i].h);   // the interposed release: uncharged
  free(v->pieces);
  v->pieces = nullptr;
  v->npieces = 0;
}

// the driver's hipMemCreate under the quota (hip mode charges here; kfd mode at the ioctl)
hipError_t real_create_charged(hipMemGenericAllocationHandle_t* handle, size_t size, const hipMemAllocationProp* prop,
                               unsigned long long flags) {
  auto f = real_hipMemCreate();
  if (!f) return hipErrorNotInitialized;
  if (!hip_active()) {
    Depth d;
    return f(handle, size, prop, flags);
  }
  uint64_t c = charge_of(size);
  if (c && !charge(c)) return deny(size);
  hipError_t e;
  {
    Depth d;
    e = f(handle, size, prop, flags);
  }
  if (e != hipSuccess || !handle) {
    uncharge(c);
    return e;
  }
  track((uint64_t)(uintptr_t)*handle, c);
  return e;
}

// with a broker arena: VMM on the device is served from it (see "VMM from the arena")
bool vmm_from_arena(const hipMemAllocationProp* prop) {
  if (!arena_configured() || t_depth || !prop || prop->type != hipMemAllocationTypePinned ||
      prop->location.type != hipMemLocationTypeDevice)
    return false;
  arena_ensure();
  return g_arena.state.load(std::memory_order_acquire) == 1 && prop->location.id == g_dev;
}

// the stand-in mapped over `p` in a window (g_arena.mu held)
VHandle* standin_at(const char* p) {
  if (!g_vva) return nullptr;
  for (uint64_t i = 0; i < kVCap; ++i) {
    uintptr_t k = g_vva[2 * i];
    if (!k || k == kTomb) continue;
    VHandle* v = reinterpret_cast<VHandle*>(g_vva[2 * i + 1]);
    if (v->at && p >= v->at && p < v->at + v->size) return v;
  }
  return nullptr;
}
}  // namespace

uint64_t vmm_slot_room_locked() {
  uint64_t room = 0;
  for (int i = 0; i < g_nwin; ++i)
    for (int s = 0; s < g_win[i].nslots; ++s)
      if (g_win[i].slot_g[s] >= 0) room += kWinAlign - g_win[i].slot_used[s];
  return room;
}

int vmm_slots_now_locked() {
  int now = 0;
  for (int i = 0; i < g_nwin; ++i)
    for (int sl = 0; sl < g_win[i].nslots; ++sl) now += g_win[i].slot_g[sl] >= 0;
  return now;
}
}  // namespace gs

using namespace gs;


GS_EXPORT hipError_t hipMemCreate(hipMemGenericAllocationHandle_t* handle, size_t size,
                                  const hipMemAllocationProp* prop, unsigned long long flags) {
  if (!real_hipMemCreate()) return hipErrorNotInitialized;
  if (handle && size && vmm_from_arena(prop)) {
    // a stand-in: its memory is decided where it is mapped (an arena slot, or the driver)
    Arena& a = g_arena;
    pthread_mutex_lock(&a.mu);
    bool ok = vtables();
    if (ok) {
      uint64_t left = 0, quota = g.quota.load();
      if (enabled() && quota) {
        uint64_t used = g.ledger->total.load();
        left = used >= quota ? 0 : quota - used;
      }
      ok = vmm_room() + left >= size;
    }
    VHandle* v = ok ? static_cast<VHandle*>(calloc(1, sizeof(VHandle))) : nullptr;
    if (v) {
      v->magic = kVHandleMagic;
      v->size = size;
      v->prop = *prop;
      v->flags = flags;
      if (!vh_put(v)) {
        free(v);
        v = nullptr;
      }
    }
    if (v) {
      g_pending_bytes += size;
      ++g_vmm_creates;
    }
    pthread_mutex_unlock(&a.mu);
    if (!v) {
      logf(1, "vmm: deny a handle of %zu bytes (arena and quota full)", size);
      return hipErrorOutOfMemory;  // what the driver says when memory is out: callers handle it
    }
    *handle = reinterpret_cast<hipMemGenericAllocationHandle_t>(v);
    return hipSuccess;
  }
  return real_create_charged(handle, size, prop, flags);
}

GS_EXPORT hipError_t hipMemAddressReserve(void** ptr, size_t size, size_t alignment, void* addr,
                                          unsigned long long flags) {
  auto f = real_hipMemAddressReserve();
  if (!f) return hipErrorNotInitialized;
  bool window = arena_configured() && !t_depth && size >= kWinAlign && !addr;
  if (window && alignment < kWinAlign) alignment = kWinAlign;  // slots on granule boundaries
  hipError_t e;
  char* vbase = nullptr;
  uint64_t vsize = size;
  {
    Depth d;
    e = f(ptr, size, alignment, addr, flags);
    vbase = e == hipSuccess && ptr ? static_cast<char*>(*ptr) : nullptr;
    if (window && vbase && reinterpret_cast<uintptr_t>(vbase) % kWinAlign) {
      // the runtime does not honour so large an alignment (HIP 7.x returns a 2 MiB-aligned range):
      // reserve one granule more and use its aligned part; the whole reservation is freed with it
      (void)real_hipMemAddressFree()(vbase, size);
      void* big = nullptr;
      if (f(&big, size + kWinAlign, 0, nullptr, flags) == hipSuccess && big) {
        vbase = static_cast<char*>(big);
        vsize = size + kWinAlign;
        *ptr = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(big) + kWinAlign - 1) & ~uintptr_t(kWinAlign - 1));
      } else {
        window = false;  // no aligned range: an ordinary reservation, its pages from the driver
        e = f(ptr, size, 0, addr, flags);
        vbase = nullptr;
      }
    }
  }
  if (e != hipSuccess || !window || !ptr || !*ptr) return e;
  pthread_mutex_lock(&g_arena.mu);
  if (g_nwin < kMaxWin) {
    Win& w = g_win[g_nwin];
    w.base = static_cast<char*>(*ptr);
    w.size = size;
    w.vbase = vbase;
    w.vsize = vsize;
    w.nslots = int((size + kWinAlign - 1) / kWinAlign);
    w.slot_g = static_cast<int32_t*>(malloc(sizeof(int32_t) * size_t(w.nslots)));
    w.slot_used = static_cast<uint64_t*>(calloc(size_t(w.nslots), sizeof(uint64_t)));
    w.slot_real = static_cast<uint32_t*>(calloc(size_t(w.nslots), sizeof(uint32_t)));
    if (w.slot_g && w.slot_used && w.slot_real) {
      for (int i = 0; i < w.nslots; ++i) w.slot_g[i] = -1;
      ++g_nwin;
    } else {
      free(w.slot_g), free(w.slot_used), free(w.slot_real);
    }
  }
  pthread_mutex_unlock(&g_arena.mu);
  return e;
}

GS_EXPORT hipError_t hipMemAddressFree(void* ptr, size_t size) {
  auto f = real_hipMemAddressFree();
  if (!f) return hipErrorNotInitialized;
  char* vbase = static_cast<char*>(ptr);
  uint64_t vsize = size;
  if (ptr && arena_configured() && !t_depth) {
    pthread_mutex_lock(&g_arena.mu);
    for (int i = 0; i < g_nwin; ++i) {
      if (g_win[i].base != ptr) continue;
      Win& w = g_win[i];
      for (int sl = 0; sl < w.nslots; ++sl)
        if (w.slot_g[sl] >= 0) slot_return(w, sl);   // pages the program never unmapped
      free(w.slot_g), free(w.slot_used), free(w.slot_real);
      vbase = w.vbase;
      vsize = w.vsize;
      g_win[i] = g_win[--g_nwin];
      break;
    }
    pthread_mutex_unlock(&g_arena.mu);
  }
  Depth d;
  return f(vbase, vsize);
}

GS_EXPORT hipError_t hipMemMap(void* ptr, size_t size, size_t offset, hipMemGenericAllocationHandle_t handle,
                               unsigned long long flags) {
  auto f = real_hipMemMap();
  if (!f) return hipErrorNotInitialized;
  if (t_depth || !arena_configured()) return f(ptr, size, offset, handle, flags);
  pthread_mutex_lock(&g_arena.mu);
  if (!vh_has(handle)) {
    pthread_mutex_unlock(&g_arena.mu);
    return f(ptr, size, offset, handle, flags);
  }
  VHandle* v = reinterpret_cast<VHandle*>(handle);
  char* va = static_cast<char*>(ptr);
  hipError_t e = hipErrorInvalidValue;
  Win* w = va && !v->at && offset == 0 && size == v->size ? win_of(va, size) : nullptr;
  if (w) {
    e = vmm_map(*w, v, va);
    if (e != hipSuccess) {
      vmm_unmap(v);
      vmm_release_pieces(v);
    } else {
      g_pending_bytes -= v->size;
      vva_put(va, v);
    }
  } else if (va && !v->at && offset == 0 && size == v->size) {
    // outside every window: the driver's memory for it, mapped where asked
    VPiece* pc = static_cast<VPiece*>(calloc(1, sizeof(VPiece)));
    if (pc) {
      e = real_create_charged(&pc->h, size, &v->prop, v->flags);
      if (e == hipSuccess) {
        Depth d;
        e = f(va, size, 0, pc->h, flags);
        if (e != hipSuccess) (void)hipMemRelease(pc->h);
      }
      if (e == hipSuccess) {
        pc->va = va;
        pc->len = size;
        v->pieces = pc;
        v->npieces = 1;
        v->at = va;
        g_pending_bytes -= v->size;
        vva_put(va, v);
        ++g_vmm_real_pieces;
      } else {
        free(pc);
      }
    } else {
      e = hipErrorOutOfMemory;
    }
  }
  pthread_mutex_unlock(&g_arena.mu);
  return e;
}

GS_EXPORT hipError_t hipMemUnmap(void* ptr, size_t size) {
  auto f = real_hipMemUnmap();
  if (!f) return hipErrorNotInitialized;
  if (t_depth || !arena_configured() || !g_vva) return f(ptr, size);
  pthread_mutex_lock(&g_arena.mu);
  // the program unmaps what it mapped, one handle's range at a time (or several at once)
  char* va = static_cast<char*>(ptr);
  char* end = va + size;
  bool any = false;
  while (va < end) {
    VHandle* v = vva_take(va);
    if (!v) break;
    any = true;
    if (win_of(v->at, v->size)) {
      vmm_unmap(v);
    } else {  // the driver piece mapped outside the windows
      Depth d;
      (void)f(v->at, v->size);
      v->at = nullptr;
    }
    va += v->size;
  }
  pthread_mutex_unlock(&g_arena.mu);
  if (any) return va == end ? hipSuccess : f(va, size_t(end - va));
  return f(ptr, size);
}

GS_EXPORT hipError_t hipMemSetAccess(void* ptr, size_t size, const hipMemAccessDesc* desc, size_t count) {
  auto f = real_hipMemSetAccess();
  if (!f) return hipErrorNotInitialized;
  if (t_depth || !arena_configured() || !ptr || !g_nwin) return f(ptr, size, desc, count);
  pthread_mutex_lock(&g_arena.mu);
  Win* w = win_of(static_cast<char*>(ptr), size);
  if (!w) {
    pthread_mutex_unlock(&g_arena.mu);
    return f(ptr, size, desc, count);
  }
  // slot by slot: the driver's memory in the range (real pages, driver pieces) gets the access
  // asked for, run by run; an arena slot is one granule mapping, read-write for this device
  // since it was backed: only access for other devices is set, on the whole granule
  bool local_rw = true;
  for (size_t k = 0; k < count; ++k)
    local_rw = local_rw && desc[k].location.type == hipMemLocationTypeDevice && desc[k].location.id == g_dev &&
               desc[k].flags == hipMemAccessFlagsProtReadWrite;
  char* lo = static_cast<char*>(ptr);
  char* hi = lo + size;
  char* run = nullptr;  // start of the current run of driver memory
  hipError_t e = hipSuccess;
  Depth d;
  auto set = [&](char* at, size_t n) {
    hipError_t r = f(at, n, desc, count);
    logf(2, "vmm: access +%llu, %zu bytes: %d", (unsigned long long)(at - w->base), n, int(r));
    if (r != hipSuccess && local_rw) {
      // HIP 7.x refuses, now and then, the access of a driver page mapped after a mapping of
      // another size in the same range, while one call over the whole run of mappings ending at
      // that page succeeds (tools/diag/vmm_spill_probe.cpp, profiles/r5/vmm_spill_probe_run*.json)
      char* from = mapped_run_start(*w, at);
      if (from < at) {
        if (auto le = real_hipGetLastError()) (void)le();
        r = f(from, size_t(at + n - from), desc, count);
        ++g_vmm_span_access;
        logf(1, "vmm: access of +%llu refused; over the run from +%llu (%llu bytes): %d",
             (unsigned long long)(at - w->base), (unsigned long long)(from - w->base),
             (unsigned long long)(at + n - from), int(r));
      }
    }
    return r;
  };
  for (char* p = lo; p < hi && e == hipSuccess;) {
    int s = int(uint64_t(p - w->base) / kWinAlign);
    char* send = w->base + uint64_t(s + 1) * kWinAlign;
    char* q = send < hi ? send : hi;
    if (w->slot_g[s] >= 0) {
      if (run) e = set(run, size_t(p - run)), run = nullptr;
      if (e == hipSuccess && !local_rw) e = set(w->base + uint64_t(s) * kWinAlign, kWinAlign);
    } else if (!run) {
      run = p;
    }
    p = q;
  }
  if (run && e == hipSuccess) e = set(run, size_t(hi - run));
  if (e != hipSuccess)
    logf(1, "vmm: access for window +%llu, %zu bytes: error %d", (unsigned long long)(lo - w->base), size, int(e));
  pthread_mutex_unlock(&g_arena.mu);
  return e;
}

GS_EXPORT hipError_t hipMemGetAllocationPropertiesFromHandle(hipMemAllocationProp* prop,
                                                             hipMemGenericAllocationHandle_t handle) {
  auto f = real_hipMemGetAllocationPropertiesFromHandle();
  if (!f) return hipErrorNotInitialized;
  if (arena_configured() && g_vh) {
    pthread_mutex_lock(&g_arena.mu);
    bool mine = vh_has(handle);
    if (mine && prop) *prop = reinterpret_cast<VHandle*>(handle)->prop;
    pthread_mutex_unlock(&g_arena.mu);
    if (mine) return prop ? hipSuccess : hipErrorInvalidValue;
  }
  return f(prop, handle);
}

GS_EXPORT hipError_t hipMemExportToShareableHandle(void* out, hipMemGenericAllocationHandle_t handle,
                                                   hipMemAllocationHandleType type, unsigned long long flags) {
  auto f = real_hipMemExportToShareableHandle();
  if (!f) return hipErrorNotInitialized;
  if (arena_configured() && g_vh) {
    pthread_mutex_lock(&g_arena.mu);
    bool mine = vh_has(handle);
    pthread_mutex_unlock(&g_arena.mu);
    // an arena page is part of a granule another pod had and will have: it is never exported
    if (mine) return hipErrorNotSupported;
  }
  return f(out, handle, type, flags);
}

GS_EXPORT hipError_t hipMemRelease(hipMemGenericAllocationHandle_t handle) {
  auto f = real_hipMemRelease();
  if (!f) return hipErrorNotInitialized;
  if (arena_configured() && g_vh) {
    pthread_mutex_lock(&g_arena.mu);
    if (vh_has(handle)) {
      VHandle* v = reinterpret_cast<VHandle*>(handle);
      if (v->retains > 0) {  // a reference hipMemRetainAllocationHandle gave out
        --v->retains;
        pthread_mutex_unlock(&g_arena.mu);
        return hipSuccess;
      }
      if (v->at) {  // released while mapped: the mapping goes with it
        char* at = v->at;
        (void)vva_take(at);
        if (win_of(at, v->size)) {
          vmm_unmap(v);
        } else if (auto un = real_hipMemUnmap()) {
          Depth d;
          (void)un(at, v->size);
          v->at = nullptr;
        }
      } else if (!v->npieces) {
        g_pending_bytes -= v->size;
      }
      vh_del(v);
      pthread_mutex_unlock(&g_arena.mu);
      vmm_release_pieces(v);
      v->magic = 0;
      free(v);
      return hipSuccess;
    }
    pthread_mutex_unlock(&g_arena.mu);
  }
  if (!hip_active()) return f(handle);
  hipError_t e;
  {
    Depth d;
    e = f(handle);
  }
  if (e == hipSuccess) uncharge(untrack((uint64_t)(uintptr_t)handle));
  return e;
}

// The handle behind a mapped address. Arena memory has none the program may hold: a hipMalloc
// block of the arena is not VMM memory to the program (invalid value, as for any hipMalloc
// pointer), and a window page is backed by the stand-in the program mapped there (returned with
// a reference that its next hipMemRelease drops). Without this the runtime would hand out the
// broker's real granule handle, which the program could then release under the arena.
GS_EXPORT hipError_t hipMemRetainAllocationHandle(hipMemGenericAllocationHandle_t* handle, void* addr) {
  auto f = real_hipMemRetainAllocationHandle();
  if (!f) return hipErrorNotInitialized;
  if (arena_configured() && addr && !t_depth) {
    if (arena_owns(addr)) return hipErrorInvalidValue;
    pthread_mutex_lock(&g_arena.mu);
    VHandle* v = standin_at(static_cast<char*>(addr));
    if (v) ++v->retains;
    pthread_mutex_unlock(&g_arena.mu);
    if (v) {
      if (handle) *handle = reinterpret_cast<hipMemGenericAllocationHandle_t>(v);
      return handle ? hipSuccess : hipErrorInvalidValue;
    }
  }
  return f(handle, addr);
}

// VMM from the arena: stand-ins created, pages mapped into arena slots, driver pieces, slots backed
// by a granule so far, and granules lent to windows now
GS_EXPORT int gpushare_shim_vmm_stats(uint64_t* creates, uint64_t* arena_maps, uint64_t* real_pieces,
                                      uint64_t* slots_backed, uint64_t* slots_now) {
  pthread_mutex_lock(&g_arena.mu);
  uint64_t now = uint64_t(vmm_slots_now_locked());
  if (creates) *creates = g_vmm_creates;
  if (arena_maps) *arena_maps = g_vmm_arena_maps;
  if (real_pieces) *real_pieces = g_vmm_real_pieces;
  if (slots_backed) *slots_backed = g_slots_backed;
  if (slots_now) *slots_now = now;
  int n = g_nwin;
  pthread_mutex_unlock(&g_arena.mu);
  return n;
}
