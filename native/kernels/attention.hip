// Flash-attention forward (prefill), bf16 in/out, fp32 softmax, causal or full, GQA.
//
// Layout: q [B, S, Hq, D], k/v [B, S, Hkv, D] with arbitrary token strides (so q/k/v can be
// slices of one fused QKV buffer), out [B, S, Hq, D] contiguous. D = 128 (or 64).
//
// Structure (cdna_hip_programming.md Appendix B "Fused attention prefill"):
//  * one workgroup = 4 waves = 64 query rows of one (batch, head); each wave owns 16 rows;
//  * K/V tiles of 64 keys, register-staged (issue global loads before the tile's compute,
//    write LDS after it: T14 split) into a 2-deep LDS ring;
//  * swapped QK^T: S^T = K * Q^T on v_mfma_f32_16x16x32_bf16, so every lane holds 16 scores
//    of ONE query row (lane & 15) -> the row max / row sum need only 2 cross-lane shuffles;
//  * O^T = V^T * P^T keeps the same lane <-> query-row mapping, so the online-softmax rescale
//    of O is lane-local; V^T fragments come from ds_read_b64_tr_b16 (T10);
//  * K rows XOR-swizzled in 16-B chunks (conflict-free ds_read_b128), V rows swizzled in
//    8-B units (conflict-free transposed reads);
//  * softmax in base 2 with the scale folded into one multiply; causal blocks scheduled
//    heaviest-first.
#include "common.h"

namespace {

constexpr int WAVES = 4, QROWS = 16 * WAVES, KT = 64;
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));

template <int D>
struct Cfg {
  static constexpr int ROWB = D * 2;              // bytes per K/V row
  static constexpr int TILEB = KT * ROWB;         // bytes per K (or V) tile
  static constexpr int STAGE = 2 * TILEB;         // K + V
  static constexpr int LDS = 2 * STAGE;           // double buffered
  static constexpr int CHUNKS = ROWB / 16;        // 16-B chunks per row
  static constexpr int LOADS = KT * CHUNKS / (WAVES * 64);  // 16-B loads per thread per tile (K or V)
};

__device__ __forceinline__ int kswz(int row, int chunk, int nchunk) { return chunk ^ (row & (nchunk - 1)); }
// V: 8-byte units, unit ^ ((row & 7) << 2)
template <int D>
__device__ __forceinline__ int vswz(int row, int unit) { return unit ^ (((row & 7) << 2) & (D / 4 - 1)); }
#define vswz_unit(r, u) vswz<D>(r, u)

// Block -> (batch*head, q-block). Workgroups are dispatched round-robin over the 8 XCDs (block i
// on XCD i mod 8), each with its own L2. Causal: q-blocks heaviest first ACROSS the whole grid
// (longest-processing-time order; a head-major order left heavy blocks of the last heads for the
// tail), and within one level the heads an XCD gets are contiguous, so the query heads sharing a
// K/V head (GQA) read it through one L2. Full attention: every XCD walks a contiguous range of
// (head, q-block), so the blocks of one head share that XCD's L2.
__device__ __forceinline__ void block_coords(int nqb, int BH, int causal, int& bh, int& qb) {
  const int i = (int)blockIdx.x;
  if (causal) {
    const int lvl = i / BH, j = i % BH;
    qb = nqb - 1 - lvl;
    bh = (BH & 7) ? j : (j & 7) * (BH >> 3) + (j >> 3);
  } else {
    const int n = BH * nqb;
    const int L = (n & 7) ? i : (i & 7) * (n >> 3) + (i >> 3);
    bh = L / nqb;
    qb = L % nqb;
  }
}

template <int D, bool TR>
__global__ __launch_bounds__(256, 2) void flash_fwd(const unsigned short* __restrict__ Q,
                                                    const unsigned short* __restrict__ K,
                                                    const unsigned short* __restrict__ V,
                                                    unsigned short* __restrict__ O, int B, int S, int Hq, int Hkv,
                                                    int q_stride, int k_stride, int v_stride, float scale_log2,
                                                    int causal) {
  using C = Cfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = (S + QROWS - 1) / QROWS;
  int bh, qb;
  block_coords(nqb, B * Hq, causal, bh, qb);
  const int b = bh / Hq, h = bh % Hq;
  const int hk = h / (Hq / Hkv);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ql = lane & 15, g = lane >> 4;
  const int q0 = qb * QROWS + wave * 16;
  const int qi = q0 + ql;                       // this lane's query row (token index)

  // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[ql][32*ds + 8g + j] ----
  bf16x8_t qf[D / 32];
  {
    const int qrow = min(qi, S - 1);
    const unsigned short* qp = Q + ((size_t)b * S + qrow) * q_stride + (size_t)h * D + 8 * g;
#pragma unroll
    for (int ds = 0; ds < D / 32; ++ds) qf[ds] = *(const bf16x8_t*)(qp + 32 * ds);
  }

  f32x4_t o[D / 16];                            // O^T tiles: lane holds O[qi][16*dt + 4g + r]
#pragma unroll
  for (int i = 0; i < D / 16; ++i) o[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  const int nkt_all = (S + KT - 1) / KT;
  const int nkt = causal ? min(nkt_all, (qb * QROWS + QROWS - 1) / KT + 1) : nkt_all;

  // ---- K/V tile staging: thread loads LOADS 16-B chunks of K and of V ----
  u16x8_t kreg[C::LOADS], vreg[C::LOADS];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int i = 0; i < C::LOADS; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / C::CHUNKS, ch = idx % C::CHUNKS;
      const int key = min(t * KT + row, S - 1);
      kreg[i] = *(const u16x8_t*)(K + ((size_t)b * S + key) * k_stride + (size_t)hk * D + ch * 8);
      vreg[i] = *(const u16x8_t*)(V + ((size_t)b * S + key) * v_stride + (size_t)hk * D + ch * 8);
    }
  };
  auto store_tile = [&](int buf) {
    char* kb = smem + buf * C::STAGE;
    char* vb = kb + C::TILEB;
#pragma unroll
    for (int i = 0; i < C::LOADS; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / C::CHUNKS, ch = idx % C::CHUNKS;
      *(u16x8_t*)(kb + row * C::ROWB + (kswz(row, ch, C::CHUNKS) << 4)) = kreg[i];
      *(u16x8_t*)(vb + row * C::ROWB + (vswz_unit(row, 2 * ch) << 3)) = vreg[i];
    }
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int t = 0; t < nkt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nkt) load_tile(t + 1);
    const char* kb = smem + cur * C::STAGE;
    const char* vb = kb + C::TILEB;

    // ---- S^T = K Q^T : 4 key sub-tiles of 16; lane holds S[qi][t*64 + 16*kt + 4g + r] ----
    f32x4_t s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int row = kt * 16 + ql;
#pragma unroll
      for (int ds = 0; ds < D / 32; ++ds) {
        const bf16x8_t kf = *(const bf16x8_t*)(kb + row * C::ROWB + (kswz(row, ds * 4 + g, C::CHUNKS) << 4));
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ds], s[kt], 0, 0, 0);
      }
    }

    // ---- online softmax (base 2), masked keys -> -inf ----
    const int kbase = t * KT + 4 * g;
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kbase + 16 * kt + r;
        float v = s[kt][r] * scale_log2;
        if (key >= S || (causal && key > qi)) v = -INFINITY;
        s[kt][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = exp2f(m - mnew);       // m = -inf on the first tile -> 0
    m = mnew;
    float psum = 0.f;
    bf16x8_t pf[2];                            // P^T fragments for the two 32-key PV steps
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[kt][r] - mnew);
        psum += p;
        pf[kt >> 1][(kt & 1) * 4 + r] = (__bf16)p;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
#pragma unroll
    for (int i = 0; i < D / 16; ++i) o[i] *= alpha;

    // ---- O^T += V^T P^T : per 32-key step s2, k(j) = 32*s2 + 4g + (j&3) + 16*(j>>2) ----
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        // lane 16g + 4q + p addresses row (rbase + q), columns 16*dt + 4p .. +3
        const int q4 = (lane & 15) >> 2, p4 = lane & 3;
        const int r0 = 32 * s2 + 4 * g + q4, r1 = r0 + 16;
        const int unit = 4 * dt + p4;
        v4s a0, a1;
        if constexpr (TR) {
          a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(vb + r0 * C::ROWB + (vswz_unit(r0, unit) << 3)));
          a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(vb + r1 * C::ROWB + (vswz_unit(r1, unit) << 3)));
        } else {  // debug path: gather the same V^T fragment element by element
          const int d = 16 * dt + ql;
          for (int e = 0; e < 4; ++e) {
            const int ra = 32 * s2 + 4 * g + e, rb = ra + 16;
            a0[e] = *(const short*)(vb + ra * C::ROWB + (vswz_unit(ra, d >> 2) << 3) + (d & 3) * 2);
            a1[e] = *(const short*)(vb + rb * C::ROWB + (vswz_unit(rb, d >> 2) << 3) + (d & 3) * 2);
          }
        }
        // whole-vector reinterpretation: element-wise bf16 inserts of the shorts miscompile
        // (hipcc emits v_perm_b32 with a repeated source register, duplicating elements)
        const v8s both = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
        const bf16x8_t vf = __builtin_bit_cast(bf16x8_t, both);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[s2], o[dt], 0, 0, 0);
      }
    }

    if (t + 1 < nkt) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: O[qi][16*dt + 4g + r] = o[dt][r] / l ----
  if (qi < S) {
    const float inv = 1.f / l;
    unsigned short* op = O + (((size_t)b * S + qi) * Hq + h) * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      u16x4_t w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = f32_to_bf16(o[dt][r] * inv);
      *(u16x4_t*)(op + 16 * dt) = w;
    }
  }
}

// ---------------------------------------------------------------------------------------
// v2 (D = 128): 8 waves x 32 query rows on v_mfma_f32_32x32x16_bf16 (256 rows per block)
//
// Same algorithm, twice the rows per wave and the 32x32 MFMA, so every K / V fragment read
// from LDS feeds twice the FLOPs of v1 (cdna_hip_programming.md "Fused attention prefill").
//  * S^T = K Q^T (A = K rows from LDS, B = Q^T in registers): lane l holds the scores of query
//    row l & 31 for keys (r & 3) + 8 (r >> 2) + 4 (l >> 5) of each 32-key sub-tile — the row
//    max / sum need one exchange with lane l ^ 32;
//  * P^T as the PV B operand: for k-step ks lane half h needs keys 16 ks + 8 h + 0..7; it holds
//    4 of them and gets the other 4 from lane l ^ 32 — one v_permlane32_swap per packed bf16
//    pair, no LDS round trip (row max / sum across the pair the same way);
//  * O^T = V^T P^T: A = V^T fragments from two ds_read_b64_tr_b16 (rows 16 ks + 8 h + 0..3 and
//    + 4..7, column 32 dt + (l & 31)); O keeps the query-row <-> lane mapping, so the online
//    rescale is lane-local;
//  * LDS images: K in 16-B chunks XOR (row & 15) (conflict-free ds_read_b128 groups), V in 8-B
//    units XOR ((row & 3) << 3) (each 32-lane tr-read group covers 32 distinct units = all 64
//    banks; 16-B staging writes stay contiguous); K/V register-staged, 2-deep ring (64 KiB);
//  * causal: only diagonal tiles are masked; waves whose rows are all above a tile skip it.
constexpr int KT8 = 64, ROW8 = 256, TILE8 = KT8 * ROW8, STAGE8 = 2 * TILE8, LDS8 = 2 * STAGE8;
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int k8swz(int row, int chunk) { return chunk ^ (row & 15); }
__device__ __forceinline__ int v8swz(int row, int unit) { return unit ^ ((row & 3) << 3); }

template <bool B>
struct BoolTag {
  static constexpr bool value = B;
};

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 (RNE): a -> low half, b -> high half
// v_permlane32_swap (probed on MI355X, tools/diag/permlane_probe.hip): r = swap(a, b) gives
// r[0] = a (lanes 0-31) | b of lane l-32 (lanes 32-63), r[1] = a of lane l+32 (lanes 0-31) | b.
__device__ __forceinline__ float pair_max(float x) {   // max over lanes l and l ^ 32
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {   // sum over lanes l and l ^ 32
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}

// Epilogue of the 32x32-MFMA kernels: lane (ql, hh) holds o[dt][4q + r] = O[row][32 dt + 8 q + 4 hh + r].
// Column group k = 4 dt + q covers columns 8k .. 8k+7, split across the half-waves; for each pair
// (2c, 2c+1) one v_permlane32_swap per dword leaves the lower half-wave with columns 16c .. 16c+7
// of its row and the upper half with 16c+8 .. 16c+15, so each lane stores 16 B per instruction
// (8 dwordx4 instead of 16 dwordx2: the store tail of the last waves is issue-bound — guide T21,
// measured +1.5-10 % on the ping-pong kernel). The swaps need all 64 lanes active: only the
// stores are predicated. `row` points at the row's first element (any valid row when !store).
__device__ __forceinline__ void store_o_wide(const f32x16_t (&o)[4], float inv, unsigned short* row, int hh,
                                             bool store) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  char* const p = (char*)row + 16 * hh;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const f32x16_t& x0 = o[c >> 1];        // groups 2c and 2c+1 share dt = c >> 1
    const int r0 = 8 * (c & 1), r1 = r0 + 4;
    const auto w0 = __builtin_amdgcn_permlane32_swap(pack_bf16x2(x0[r0] * inv, x0[r0 + 1] * inv),
                                                     pack_bf16x2(x0[r1] * inv, x0[r1 + 1] * inv), false, false);
    const auto w1 = __builtin_amdgcn_permlane32_swap(pack_bf16x2(x0[r0 + 2] * inv, x0[r0 + 3] * inv),
                                                     pack_bf16x2(x0[r1 + 2] * inv, x0[r1 + 3] * inv), false, false);
    if (store) *(u32x4_t*)(p + 32 * c) = u32x4_t{w0[0], w1[0], w0[1], w1[1]};
  }
}

// NW waves per block (NW x 32 query rows). NW = 4 runs two independent blocks per CU (their
// per-tile barriers drift apart, so one block's softmax overlaps the other's MFMAs); NW = 8 is
// one block per CU.
constexpr float RESCALE_TAU = 8.f;   // log2 units: deferred-rescale headroom (p <= 256)

// FLAGS bit 0 (PRIO): the younger half of an 8-wave block runs at s_setprio 1 (it loses every
// VALU arbitration to its older SIMD partner otherwise); bit 1 (LATE): tile t+2's global loads are
// issued after QK^T(t) and written to LDS right after the next barrier (T14 split: the staging
// registers are not live across QK^T), instead of loads at the tile's start and the LDS write
// before its closing barrier.
// AF_WIDE: the widened epilogue (store_o_wide) on the 4-wave block; the 8-wave block always uses
// it. On the 4-wave block at the 256-register budget it costs 3 spilled registers (A/B: variant 13).
enum { AF_PRIO = 1, AF_LATE = 2, AF_WIDE = 4 };

template <int NW, int FLAGS = 0>
__global__ __launch_bounds__(NW * 64, 8 / NW) void flash_fwd_d128_w8(const unsigned short* __restrict__ Q,
                                                            const unsigned short* __restrict__ K,
                                                            const unsigned short* __restrict__ V,
                                                            unsigned short* __restrict__ O, int B, int S, int Hq,
                                                            int Hkv, int q_stride, int k_stride, int v_stride,
                                                            float scale_log2, int causal) {
  constexpr int QR8 = 32 * NW, NT = NW * 64, LD = 1024 / NT;   // 16-B staging loads per thread (K or V)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = (S + QR8 - 1) / QR8;
  int bh, qb;
  block_coords(nqb, B * Hq, causal, bh, qb);
  const int b = bh / Hq, h = bh % Hq;
  const int hk = h / (Hq / Hkv);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ql = lane & 31, hh = lane >> 5;
  const int q0 = qb * QR8 + wave * 32;
  const int qi = q0 + ql;
  constexpr bool LATE = (FLAGS & AF_LATE) != 0;
  if constexpr ((FLAGS & AF_PRIO) != 0 && NW == 8) {
    // wave-uniform branch (readfirstlane), so the scalar s_setprio is guarded per wave
    if (__builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }

  // Q^T fragments (B operand): lane holds Q[qi][16 ds + 8 hh + j]
  bf16x8_t qf[8];
  {
    const unsigned short* qp = Q + ((size_t)b * S + min(qi, S - 1)) * q_stride + (size_t)h * 128 + 8 * hh;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) qf[ds] = *(const bf16x8_t*)(qp + 16 * ds);
  }
  f32x16_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = -INFINITY, l = 0.f;

  const int nkt_all = (S + KT8 - 1) / KT8;
  const int nkt = causal ? min(nkt_all, (qb * QR8 + QR8 - 1) / KT8 + 1) : nkt_all;

  // register staging: 1024 16-B chunks per K (or V) tile / NT threads
  u16x8_t kreg[LD], vreg[LD];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int idx = tid + i * NT, row = idx >> 4, ch = idx & 15;
      const int key = min(t * KT8 + row, S - 1);
      kreg[i] = *(const u16x8_t*)(K + ((size_t)b * S + key) * k_stride + (size_t)hk * 128 + ch * 8);
      vreg[i] = *(const u16x8_t*)(V + ((size_t)b * S + key) * v_stride + (size_t)hk * 128 + ch * 8);
    }
  };
  auto store_tile = [&](int buf) {
    char* kb = smem + buf * STAGE8;
    char* vb = kb + TILE8;
#pragma unroll
    for (int i = 0; i < LD; ++i) {
      const int idx = tid + i * NT, row = idx >> 4, ch = idx & 15;
      *(u16x8_t*)(kb + row * ROW8 + (k8swz(row, ch) << 4)) = kreg[i];
      *(u16x8_t*)(vb + row * ROW8 + (v8swz(row, 2 * ch) << 3)) = vreg[i];
    }
  };

  load_tile(0);
  store_tile(0);
  if (LATE && nkt > 1) load_tile(1);
  __syncthreads();

  for (int t = 0; t < nkt; ++t) {
    const int cur = t & 1;
    if constexpr (LATE) {
      if (t + 1 < nkt) store_tile(cur ^ 1);     // tile t+1 (loaded during t-1): its buffer was freed by the barrier
    } else {
      if (t + 1 < nkt) load_tile(t + 1);
    }
    auto prefetch = [&]() {
      if constexpr (LATE) {
        if (t + 2 < nkt) load_tile(t + 2);
      }
    };
    const char* kb = smem + cur * STAGE8;
    const char* vb = kb + TILE8;
    const int kfirst = t * KT8;
    const bool active = !causal || kfirst <= q0 + 31;           // some key of the tile is visible
    // The tile body is instantiated twice (diagonal/ragged tiles with the mask, the rest without)
    // so each path is one basic block the scheduler can interleave (softmax VALU under MFMAs).
    auto body = [&](auto tag) {
      constexpr bool MASKED = decltype(tag)::value;
      // ---- S^T = K Q^T, two 32-key sub-tiles ----
      f32x16_t s[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[st][r] = 0.f;
        const int row = 32 * st + ql;
#pragma unroll
        for (int ds = 0; ds < 8; ++ds) {
          const bf16x8_t kf = *(const bf16x8_t*)(kb + row * ROW8 + (k8swz(row, 2 * ds + hh) << 4));
          s[st] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ds], s[st], 0, 0, 0);
        }
      }
      prefetch();
      // ---- online softmax (base 2); masking only on diagonal / ragged tiles ----
      // The max is taken on the raw scores (scale > 0) and the scale folded into one FMA per
      // score: p = 2^(s * scale - m). Deferred rescale (T13): the running max m moves only when
      // a tile's max exceeds it by more than RESCALE_TAU (p then stays <= 2^TAU, harmless in
      // fp32 and in bf16's relative precision), so the 64-register O rescale and l's multiply
      // run only on the few tiles where some row's max really grows — the decision is
      // wave-uniform and O, l see the same factor, before this tile's P V.
      float tmax = -INFINITY;
      if constexpr (MASKED) {
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kfirst + 32 * st + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const float v = (key >= S || (causal && key > qi)) ? -INFINITY : s[st][r];
            s[st][r] = v;
            tmax = fmaxf(tmax, v);
          }
      } else {
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, s[st][r]);
      }
      tmax = pair_max(tmax) * scale_log2;
      const bool grow = tmax > m + RESCALE_TAU;
      if (__builtin_amdgcn_ballot_w64(grow)) {
        const float mnew = grow ? tmax : m;
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);   // raw v_exp_f32 (exp2(-inf) = 0)
        m = mnew;
        l *= alpha;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] *= alpha;
      }
      const float mneg = -m;
      float psum = 0.f;
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[st][r], scale_log2, mneg));
          s[st][r] = pv;
          psum += pv;
        }
      l += pair_sum(psum);

      // ---- O^T += V^T P^T over 4 k-steps of 16 keys ----
      const int g16 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        // the two 4-key blocks of this k-step at compile-time register indices: lo = keys
        // base + 4 hh + 0..3, hi = base + 8 + 4 hh + 0..3 (base = 16 (ks & 1) in the sub-tile)
        const int st = ks >> 1, rb = 8 * (ks & 1);
        const unsigned lo0 = pack_bf16x2(s[st][rb + 0], s[st][rb + 1]);
        const unsigned lo1 = pack_bf16x2(s[st][rb + 2], s[st][rb + 3]);
        const unsigned hi0 = pack_bf16x2(s[st][rb + 4], s[st][rb + 5]);
        const unsigned hi1 = pack_bf16x2(s[st][rb + 6], s[st][rb + 7]);
        // half 0 needs {own lo, partner's lo}, half 1 {partner's hi, own hi}: swap(lo, hi) returns
        // exactly those two words in that order on both halves — no select, no LDS round trip
        const auto w0 = __builtin_amdgcn_permlane32_swap(lo0, hi0, false, false);
        const auto w1 = __builtin_amdgcn_permlane32_swap(lo1, hi1, false, false);
        typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
        const u32x4_t pw = u32x4_t{w0[0], w1[0], w0[1], w1[1]};
        const bf16x8_t pf = __builtin_bit_cast(bf16x8_t, pw);
        // V^T fragment rows (keys) 16 ks + 8 hh + {0..3 | 4..7}; lane (4 q4 + p4) of its 16-lane
        // group addresses row q4, columns 4 p4 .. 4 p4 + 3 of the group's 16-column block
        const int r0 = 16 * ks + 8 * (g16 >> 1) + q4, r1 = r0 + 4;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int unit = 8 * dt + 4 * (g16 & 1) + p4;
          const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(vb + r0 * ROW8 + (v8swz(r0, unit) << 3)));
          const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(vb + r1 * ROW8 + (v8swz(r1, unit) << 3)));
          const v8s both = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, both), pf, o[dt], 0, 0, 0);
        }
      }
    };
    if (active) {
      if ((causal && kfirst + KT8 - 1 > q0) || kfirst + KT8 > S)
        body(BoolTag<true>{});
      else
        body(BoolTag<false>{});
    } else {
      prefetch();
    }
    if (!LATE && t + 1 < nkt) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: O[qi][32 dt + 8 (r >> 2) + 4 hh + (r & 3)] = o[dt][r] / l ----
  if constexpr (NW == 8 || (FLAGS & AF_WIDE) != 0) {
    store_o_wide(o, 1.f / l, O + (((size_t)b * S + min(qi, S - 1)) * Hq + h) * 128, hh, qi < S);
  } else if (qi < S) {
    const float inv = 1.f / l;
    unsigned short* op = O + (((size_t)b * S + qi) * Hq + h) * 128 + 4 * hh;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u16x4_t w;
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = f32_to_bf16(o[dt][4 * q + r] * inv);
        *(u16x4_t*)(op + 32 * dt + 8 * q) = w;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Ping-pong 8-wave kernel (D = 128): the two waves that share a SIMD run in antiphase.
//
// In the kernels above the 8 waves of a CU meet at one barrier per K/V tile and then all do the
// same thing: QK^T (matrix pipe contended, VALU idle), softmax (VALU busy, matrix pipe idle), PV.
// Here each wave software-pipelines its tile loop into two segments — an MFMA segment
// M(j) = { O += V(j-1)^T P(j-1)^T ; S(j) = K(j) Q^T } (32 MFMAs) and a VALU segment
// V(j) = { softmax(S(j)) -> P(j), O/l rescale } — and the younger half (waves 4-7) runs one
// segment behind the older half (waves 0-3). One workgroup barrier closes every segment, so in
// every segment each SIMD has one wave on the matrix pipe and its partner on the VALU:
//
//   global segment   0      1      2      3      4   ...
//   waves 0-3        M(0)   V(0)   M(1)   V(1)   M(2)
//   waves 4-7        -      M(0)   V(0)   M(1)   V(1)
//
// K(j) and V(j-1) are read during global segments 2j and 2j+1, so a 2-deep ring for K and one for
// V (64 KiB) suffices. K(i+1) and V(i) arrive by LDS DMA (buffer_load ... lds, 1 KiB per wave
// instruction, 2+2 per wave per tile) issued at the start of segment 2i into the buffers K(i-1) /
// V(i-2) left after segment 2i-1, and are waited for (vmcnt) before the barrier closing segment
// 2i+1 — two segments of latency cover, no staging registers, no LDS store instructions. The
// XOR swizzles are applied on the source side (lane-linear LDS image). P(j) (16 packed registers)
// carries from V(j) to M(j+1); S(j) (32) from M(j) to V(j). Inside M(j) the 32 MFMAs run in 4
// groups (PV k-step g with 4 of QK's), each group's 8 V^T + 4 K fragment reads issued one group
// ahead.
template <bool PV, bool QK>
struct MSegTag {
  static constexpr bool pv = PV, qk = QK;
};

// PP_PRIO: the wave in its MFMA segment runs at s_setprio 1, so its MFMA / LDS issue wins the
// arbitration against the partner's softmax VALU stream.
// PP_ILV: SIMD partners take neighbouring 32-row slices (see q0 below) instead of rows 32 w and
// 32 w + 128.
// PP_TRACE (diagnostics, tools/attn_trace.py): block 0's waves record s_memtime before and after
// every segment barrier into g_pp_trace (vector stores from lane 0).
// PP_WIDE: the epilogue pairs column groups across the half-waves (v_permlane32_swap) so each
// lane stores 16 B per instruction: 8 dwordx4 stores per lane instead of 16 dwordx2 (the store
// tail of the last-finishing waves is issue-bound, not HBM-bound).
// PP_SPRIO: static priority instead of PP_PRIO's per-segment flips — the younger half (waves
// 4-7, which lose VALU arbitration to the older half by age) runs at s_setprio 1 throughout.
enum { PP_PRIO = 1, PP_ILV = 2, PP_TRACE = 4, PP_WIDE = 8, PP_SPRIO = 16 };
constexpr int PP_TRACE_SEGS = 160;
__device__ unsigned long long g_pp_trace[8][PP_TRACE_SEGS][2];

template <int FLAGS = 0>
__global__ __launch_bounds__(512, 1) void flash_fwd_d128_pp(const unsigned short* __restrict__ Q,
                                                           const unsigned short* __restrict__ K,
                                                           const unsigned short* __restrict__ V,
                                                           unsigned short* __restrict__ O, int B, int S, int Hq,
                                                           int Hkv, int q_stride, int k_stride, int v_stride,
                                                           float scale_log2, int causal) {
  constexpr int NW = 8, QR8 = 32 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kbuf = smem;                 // K ring: 2 x TILE8
  char* const vbuf = smem + 2 * TILE8;     // V ring: 2 x TILE8
  const int nqb = (S + QR8 - 1) / QR8;
  int bh, qb;
  block_coords(nqb, B * Hq, causal, bh, qb);
  const int b = bh / Hq, h = bh % Hq;
  const int hk = h / (Hq / Hkv);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2;              // 0: waves 0-3, 1: waves 4-7
  const int ql = lane & 31, hh = lane >> 5;
  // rows: the SIMD partners (wave w of each half) take neighbouring 32-row slices, so under a
  // causal mask both have (almost) the same number of live tiles and stay in antiphase to the end
  const int q0 = qb * QR8 + ((FLAGS & PP_ILV) ? (wave & 3) * 64 + half * 32 : wave * 32);
  const int qi = q0 + ql;

  bf16x8_t qf[8];
  {
    const unsigned short* qp = Q + ((size_t)b * S + min(qi, S - 1)) * q_stride + (size_t)h * 128 + 8 * hh;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) qf[ds] = *(const bf16x8_t*)(qp + 16 * ds);
  }
  f32x16_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  f32x16_t sacc[2];
  bf16x8_t pf[4];

  const int nkt_all = (S + KT8 - 1) / KT8;
  const int nkt = causal ? min(nkt_all, (qb * QR8 + QR8 - 1) / KT8 + 1) : nkt_all;

  // ---- LDS DMA: instruction i (0, 1) of wave w fills rows 32 i + 4 w + lane / 16 of a tile;
  // lane's 16-B slot lane & 15 receives the logical chunk the swizzle puts there (the XOR terms
  // depend on row & 15 / row & 3 only, the same for both i). Rows past S read as zeros (buffer
  // range check); their scores are masked and their P is 0.
  const int prow = 4 * wave + (lane >> 4);
  const int kch = (lane & 15) ^ (prow & 15);
  const int vch = (lane & 15) ^ ((prow & 3) << 2);
  const __amdgpu_buffer_rsrc_t rK = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(K + (size_t)b * S * k_stride + (size_t)hk * 128), (short)0, S * k_stride * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rV = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(V + (size_t)b * S * v_stride + (size_t)hk * 128), (short)0, S * v_stride * 2, 0x00020000);
  const unsigned voffK = (unsigned)(prow * k_stride + kch * 8) * 2u;
  const unsigned voffV = (unsigned)(prow * v_stride + vch * 8) * 2u;
  auto dma_k = [&](int t, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rK, (__attribute__((address_space(3))) void*)(kbuf + buf * TILE8 + i * 8192 + wave * 1024), 16, voffK,
          (t * KT8 + 32 * i) * k_stride * 2, 0, 0);
  };
  auto dma_v = [&](int t, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rV, (__attribute__((address_space(3))) void*)(vbuf + buf * TILE8 + i * 8192 + wave * 1024), 16, voffV,
          (t * KT8 + 32 * i) * v_stride * 2, 0, 0);
  };
  // a tile is live for this wave when some key of it is visible to some row of the wave
  auto live = [&](int t) __attribute__((always_inline)) { return !causal || t * KT8 <= q0 + 31; };

  // ---- M segment: 8 sub-groups of 4 MFMAs — PV k-step g (4 V^T fragments) alternating with
  // QK quarter g (sub-tile g >> 1, d-steps 4 (g & 1) .. +3: 4 K fragments); each sub-group's
  // 4 fragments (16 registers) are read one sub-group ahead
  struct Frag {
    bf16x8_t x[4];
  };
  auto mseg = [&](int jp, int jq, auto tag, auto after_reads) __attribute__((always_inline)) {
    constexpr bool DO_PV = decltype(tag)::pv, DO_QK = decltype(tag)::qk;
    constexpr int NSUB = (DO_PV ? 4 : 0) + (DO_QK ? 4 : 0);
    // fragment addresses are recomputed here from an opaque copy of the lane id (a few VALU on
    // an otherwise matrix-bound segment) instead of being hoisted out of the loop: 12 per-lane
    // XOR offsets kept live across the loop spilled, and a spill reload's vmcnt(0) also waits
    // for the in-flight K/V DMA
    int lx = lane;
    asm volatile("" : "+v"(lx));
    const int g16 = lx >> 4, q4 = (lx & 15) >> 2, p4 = lx & 3, ql = lx & 31, hh = lx >> 5;
    const char* vb = vbuf + (jp & 1) * TILE8;
    const char* kb = kbuf + (jq & 1) * TILE8;
    // sub-group u: PV step when (DO_PV and (u even or !DO_QK)), else QK quarter
    auto is_pv = [&](int u) __attribute__((always_inline)) { return DO_PV && (!DO_QK || (u & 1) == 0); };
    auto step = [&](int u) __attribute__((always_inline)) { return (DO_PV && DO_QK) ? (u >> 1) : u; };
    auto rd = [&](Frag& f, int u) __attribute__((always_inline)) {
      const int g = step(u);
      if (is_pv(u)) {
        const int r0 = 16 * g + 8 * (g16 >> 1) + q4, r1 = r0 + 4;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int unit = 8 * dt + 4 * (g16 & 1) + p4;
          const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(vb + r0 * ROW8 + (v8swz(r0, unit) << 3)));
          const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(vb + r1 * ROW8 + (v8swz(r1, unit) << 3)));
          f.x[dt] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      } else {
        const int row = 32 * (g >> 1) + ql;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int ds = 4 * (g & 1) + d;
          f.x[d] = *(const bf16x8_t*)(kb + row * ROW8 + (k8swz(row, 2 * ds + hh) << 4));
        }
      }
    };
    auto mm = [&](const Frag& f, int u) __attribute__((always_inline)) {
      const int g = step(u);
      if (is_pv(u)) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.x[dt], pf[g], o[dt], 0, 0, 0);
      } else {
        const int st = g >> 1;
        if ((g & 1) == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc[st][r] = 0.f;
        }
#pragma unroll
        for (int d = 0; d < 4; ++d)
          sacc[st] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.x[d], qf[4 * (g & 1) + d], sacc[st], 0, 0, 0);
      }
    };
    if constexpr ((FLAGS & PP_PRIO) != 0) __builtin_amdgcn_s_setprio(1);
    Frag f[2];
    rd(f[0], 0);
#pragma unroll
    for (int u = 0; u < NSUB; ++u) {
      if (u + 1 < NSUB) rd(f[(u + 1) & 1], u + 1);
      if (u + 2 == NSUB) {
        // after the segment's last fragment read: the compiler makes every LDS read that
        // follows an LDS DMA wait for it (vmcnt), so DMAs are issued behind the reads
        __builtin_amdgcn_sched_barrier(0);
        after_reads();
      }
      __builtin_amdgcn_sched_barrier(0);
      mm(f[u & 1], u);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr ((FLAGS & PP_PRIO) != 0) __builtin_amdgcn_s_setprio(0);
  };
  auto nop = [&]() __attribute__((always_inline)) {};
  auto softmax = [&](int j, auto tag) __attribute__((always_inline)) {
    constexpr bool MASKED = decltype(tag)::value;
    const int kfirst = j * KT8;
    float tmax = -INFINITY;
    if constexpr (MASKED) {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kfirst + 32 * st + (r & 3) + 8 * (r >> 2) + 4 * hh;
          const float v = (key >= S || (causal && key > qi)) ? -INFINITY : sacc[st][r];
          sacc[st][r] = v;
          tmax = fmaxf(tmax, v);
        }
    } else {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sacc[st][r]);
    }
    tmax = pair_max(tmax) * scale_log2;
    const bool grow = tmax > m + RESCALE_TAU;
    if (__builtin_amdgcn_ballot_w64(grow)) {      // O is idle here: PV(j-1) finished in M(j)
      const float mnew = grow ? tmax : m;
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      m = mnew;
      l *= alpha;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] *= alpha;
    }
    // the softmax segment is the long pole of the ping-pong pair (tools/attn_trace.py). Packed
    // v_pk_fma/v_pk_add here slowed the partner's MFMA segment by ~600 cycles (measured), and
    // 4 independent sum/max chains did not shorten the segment: plain single ops, one chain
    const float mneg = -m;
    float psum = 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pvv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[st][r], scale_log2, mneg));
        sacc[st][r] = pvv;
        psum += pvv;
      }
    l += pair_sum(psum);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int st = ks >> 1, rb = 8 * (ks & 1);
      const unsigned lo0 = pack_bf16x2(sacc[st][rb + 0], sacc[st][rb + 1]);
      const unsigned lo1 = pack_bf16x2(sacc[st][rb + 2], sacc[st][rb + 3]);
      const unsigned hi0 = pack_bf16x2(sacc[st][rb + 4], sacc[st][rb + 5]);
      const unsigned hi1 = pack_bf16x2(sacc[st][rb + 6], sacc[st][rb + 7]);
      const auto w0 = __builtin_amdgcn_permlane32_swap(lo0, hi0, false, false);
      const auto w1 = __builtin_amdgcn_permlane32_swap(lo1, hi1, false, false);
      typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
      pf[ks] = __builtin_bit_cast(bf16x8_t, u32x4_t{w0[0], w1[0], w0[1], w1[1]});
    }
  };

  auto dma_pair = [&](int i) __attribute__((always_inline)) {              // K(i+1), V(i) -> the buffers freed after segment 2i-1
    if (i + 1 < nkt) dma_k(i + 1, (i + 1) & 1);
    if (i < nkt) dma_v(i, i & 1);
  };
  // Segment barrier without __syncthreads' release/acquire fences: the release fence would make
  // every barrier wait for this wave's in-flight LDS DMA (vmcnt(0)), which must instead overlap
  // a whole segment. LDS reads are consumed (lgkmcnt) inside their segment, so the only
  // ordering a barrier needs is the DMA one, waited for explicitly at odd segments; the empty
  // asm with a memory clobber keeps the compiler from moving LDS accesses across it.
  int tseg = 0;
  const bool tracer = (FLAGS & PP_TRACE) && blockIdx.x == 0 && lane == 0;
  auto bar = [&]() __attribute__((always_inline)) {
    if constexpr ((FLAGS & PP_TRACE) != 0) {
      if (tracer && tseg < PP_TRACE_SEGS) g_pp_trace[wave][tseg][0] = __builtin_amdgcn_s_memtime();
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if constexpr ((FLAGS & PP_TRACE) != 0) {
      ++tseg;
      if (tracer && tseg < PP_TRACE_SEGS) g_pp_trace[wave][tseg][1] = __builtin_amdgcn_s_memtime();
    }
  };
  auto wait_sync = [&]() __attribute__((always_inline)) {   // closes an odd segment: this wave's DMAs landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
  };
  auto needmask = [&](int j) __attribute__((always_inline)) { return (causal && j * KT8 + KT8 - 1 > q0) || j * KT8 + KT8 > S; };
  auto smax_any = [&](int j) __attribute__((always_inline)) {
    if (needmask(j))
      softmax(j, BoolTag<true>{});
    else
      softmax(j, BoolTag<false>{});
  };
  // tiles 0 .. nlive-1 hold a key visible to this wave; only the last of them can need the mask
  // (causal diagonal or ragged end). Later tiles are only staged and waited for, so both halves
  // meet 2 nkt + 2 barriers with straight-line loop bodies (no per-segment branches whose merges
  // made the compiler shuffle O and S between register sets).
  const int nlive = causal ? min(nkt, (q0 + 31) / KT8 + 1) : nkt;

  if constexpr ((FLAGS & PP_SPRIO) != 0) {
    if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);   // wave-uniform guard
  }
  // ---- prologue: K(0) in LDS ----
  dma_k(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();

  if (half == 0) {
    // waves 0-3: M(j) in segment 2j, V(j) in segment 2j+1; DMA issued behind M(j)'s reads
    mseg(0, 0, MSegTag<false, true>{}, [&]() __attribute__((always_inline)) { dma_pair(0); });
    bar();
    smax_any(0);
    wait_sync();
    int j = 1;
    for (; j < nlive - 1; ++j) {
      mseg(j - 1, j, MSegTag<true, true>{}, [&]() __attribute__((always_inline)) { dma_pair(j); });
      bar();
      softmax(j, BoolTag<false>{});
      wait_sync();
    }
    if (j == nlive - 1) {
      mseg(j - 1, j, MSegTag<true, true>{}, [&]() __attribute__((always_inline)) { dma_pair(j); });
      bar();
      smax_any(j);
      wait_sync();
      ++j;
    }
    mseg(j - 1, 0, MSegTag<true, false>{}, [&]() __attribute__((always_inline)) { dma_pair(j); });  // j == nlive
    bar();
    wait_sync();
    for (++j; j <= nkt; ++j) {
      dma_pair(j);
      bar();
      wait_sync();
    }
  } else {
    // waves 4-7: V(j-1) in segment 2j, M(j) in segment 2j+1
    dma_pair(0);
    bar();
    mseg(0, 0, MSegTag<false, true>{}, nop);
    wait_sync();
    int j = 1;
    for (; j < nlive; ++j) {
      dma_pair(j);
      softmax(j - 1, BoolTag<false>{});        // j - 1 < nlive - 1: never masked
      bar();
      mseg(j - 1, j, MSegTag<true, true>{}, nop);
      wait_sync();
    }
    dma_pair(j);                              // j == nlive: V(nlive-1), the last PV
    smax_any(j - 1);
    bar();
    mseg(j - 1, 0, MSegTag<true, false>{}, nop);
    wait_sync();
    for (++j; j <= nkt; ++j) {
      dma_pair(j);
      bar();
      wait_sync();
    }
  }

  if constexpr ((FLAGS & PP_WIDE) != 0) {
    store_o_wide(o, 1.f / l, O + (((size_t)b * S + min(qi, S - 1)) * Hq + h) * 128, hh, qi < S);
  } else if (qi < S) {
    const float inv = 1.f / l;
    unsigned short* op = O + (((size_t)b * S + qi) * Hq + h) * 128 + 4 * hh;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u16x4_t w;
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = f32_to_bf16(o[dt][4 * q + r] * inv);
        *(u16x4_t*)(op + 32 * dt + 8 * q) = w;
      }
  }
}

template <int FLAGS = 0>
int launch_pp(const void* q, const void* k, const void* v, void* o, int B, int S, int Hq, int Hkv, int qs, int ks,
              int vs, float scale_log2, int causal, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)flash_fwd_d128_pp<FLAGS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8);
    attr = true;
  }
  const int nqb = (S + 255) / 256;
  flash_fwd_d128_pp<FLAGS><<<dim3((unsigned)(B * Hq * nqb)), dim3(512), LDS8, stream>>>(
      (const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v, (unsigned short*)o, B, S, Hq,
      Hkv, qs, ks, vs, scale_log2, causal & 1);
  return gs_launch_status();
}

// ---------------------------------------------------------------------------------------------
// One wave per SIMD, 64 query rows per wave (D = 128): flash_fwd_d128_w64.
//
// The ping-pong kernel above pairs two 32-row waves per SIMD in antiphase; its softmax segment
// (~1800 cycles, VALU-issue bound) sets the pace while the partner's 32 MFMAs take ~1300, so the
// matrix pipe idles a third of the time (profiles/attention_r2.md). Here a single wave per SIMD
// owns 64 rows and interleaves its own softmax of tile j into the issue gaps of its MFMA stream
// {P·V(j-1), QK^T(j+1)}: a v_mfma_f32_32x32x16_bf16 holds the SIMD's vector issue for 8 of its
// 32 cycles (MI355X_MICROARCH.md, issue-cost row), so ~24 cycles of VALU per MFMA ride along.
//
// Tiles are 32 keys: per tile a wave issues 32 MFMAs (16 P·V + 16 QK^T, 1024 matrix cycles)
// beside ~700 cycles of softmax issue for its 64 x 32 scores. Registers (512 per lane at one
// wave per SIMD): Q^T (16 bf16x8 fragments, 64) and P (16) live in AGPRs and are read by the
// MFMAs from there (every MFMA is inline asm with "a" B operands); O^T (8 tiles of 32x32 fp32,
// 128), S^T of the tile being softmaxed and of the tile being produced (2 x 32), one fragment set
// and the 12 per-lane LDS offsets are VGPRs. O stays out of the AGPRs on purpose: the rare
// online-softmax rescale is a branch, and an accumulator whose value merges at a branch join was
// copied AGPR -> VGPR by the allocator on every iteration (measured in the .s); 64-key tiles
// (2 x 64 S registers) spilled Q to scratch. The two S buffers alternate by name (the loop is
// unrolled by two), never by a runtime index; one P buffer suffices (P(j-1) is consumed in the
// first half of iteration j, P(j) produced in its second half).
//
// Lane mapping (swapped QK^T, as the other 32x32 kernels): lane (ql, hh) holds query rows
// q0 + ql (block c = 0) and q0 + 32 + ql (c = 1); S^T tile c register r is key
// 8 (r >> 2) + 4 hh + (r & 3) of the tile; O^T tile (c, dt) register r is dim 32 dt + 8 (r >> 2) +
// 4 hh + (r & 3).
//
// K/V tiles arrive by LDS DMA issued from inline asm (the compiler would otherwise make every
// later LDS read of the iteration wait for the DMA, vmcnt): K(j+2) and V(j) at the start of
// iteration j into the slots iteration j-1 finished reading, waited for (vmcnt(0)) before the one
// raw barrier that opens iteration j+1 — a whole iteration of latency cover. Hazards the compiler
// does not see around asm are padded by hand: MFMA results are read by VALU only an iteration
// later or after explicit s_nop, and AGPR writes are padded before the next MFMA reads them.
constexpr int W64_QR = 256;                 // rows per block: 4 waves x 64
// diagnostics: compiler-issued LDS DMA (waits for it at every LDS read); a 64-cycle pad after every
// MFMA group
// timing-only diagnostics (wrong results): no iteration barrier / no in-step DMA
// W64_REGSTAGE: the step's K/V tiles come through AGPRs (buffer_load into AGPRs in the first work
// slots, ds_write_b128 from them at the step's end) instead of LDS DMA, whose issue costs ~60
// cycles a piece beside MFMAs (measured: the in-step DMA was 15 % of the kernel's time)
enum { W64_BUILTIN_DMA = 1, W64_PAD = 2, W64_T_NOBAR = 4, W64_T_NODMA = 8, W64_REGSTAGE = 16 };
constexpr int W64_KT = 32, W64_TILE = W64_KT * ROW8, W64_LDS = 4 * W64_TILE;

typedef int i32x4_t __attribute__((ext_vector_type(4)));

template <int I>
struct W64Int {
  static constexpr int value = I;
};
template <int B, int E, typename F>
__device__ __forceinline__ void w64_static_for(F&& f) {
  if constexpr (B < E) {
    f(W64Int<B>{});
    w64_static_for<B + 1, E>(f);
  }
}

template <bool PV, bool SM, bool QK, bool MASK>
struct W64Tag {
  static constexpr bool pv = PV, sm = SM, qk = QK, mask = MASK;
};

// Inline asm (operands in the register files chosen here), so the compiler does not see the MFMA
// latency: a copy of an accumulator tuple placed right after the MFMA that writes it would read
// rows the MFMA has not written yet (measured: stale upper halves of O tiles). Every place the
// allocator may copy — block boundaries — is therefore preceded by a pad: the end of each step
// and the start of each iteration (open), and no branch sits between MFMAs.
#define W64_MFMA_QK0(d, k, q) \
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(k), "a"(q))
#define W64_MFMA_QK(d, k, q) \
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(k), "a"(q))
#define W64_MFMA_PV(o, v, p) \
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o) : "v"(v), "a"(p))

template <int FLAGS = 0>
__global__ __launch_bounds__(256, 1) void flash_fwd_d128_w64(const unsigned short* __restrict__ Q,
                                                            const unsigned short* __restrict__ K,
                                                            const unsigned short* __restrict__ V,
                                                            unsigned short* __restrict__ O, int B, int S, int Hq,
                                                            int Hkv, int q_stride, int k_stride, int v_stride,
                                                            float scale_log2, int causal) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kbuf = smem;                   // K ring: 2 x W64_TILE
  char* const vbuf = smem + 2 * W64_TILE;    // V ring: 2 x W64_TILE
  const int nqb = (S + W64_QR - 1) / W64_QR;
  int bh, qb;
  block_coords(nqb, B * Hq, causal, bh, qb);
  const int b = bh / Hq, h = bh % Hq;
  const int hk = h / (Hq / Hkv);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ql = lane & 31, hh = lane >> 5;
  const int q0 = qb * W64_QR + wave * 64;

  // ---- Q^T fragments (B operand), pinned in AGPRs: qf[c][ds] = Q[q0 + 32 c + ql][16 ds + 8 hh ..]
  bf16x8_t qf[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const unsigned short* qp =
        Q + ((size_t)b * S + min(q0 + 32 * c + ql, S - 1)) * q_stride + (size_t)h * 128 + 8 * hh;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) qf[c][ds] = *(const bf16x8_t*)(qp + 16 * ds);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) asm volatile("" : "+a"(qf[c][ds]));
  f32x16_t o[2][4];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) o[c][dt][r] = 0.f;
      asm volatile("" : "+a"(o[c][dt]));
    }
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  f32x16_t sA[2], sB[2];
  bf16x8_t pP[2][2];                          // [c][g]: P^T of 16-key step g

  const int nkt_all = (S + W64_KT - 1) / W64_KT;
  const int nkt = causal ? min(nkt_all, (qb * W64_QR + W64_QR - 1) / W64_KT + 1) : nkt_all;
  // tiles 0 .. nlive-1 hold a key visible to this wave; causal: the last two straddle the
  // diagonal, ragged S: the last one is partial
  const int nlive = causal ? min(nkt, (q0 + 63) / W64_KT + 1) : nkt;
  const int mask_from = causal ? nlive - 2 : ((S % W64_KT) ? nlive - 1 : nlive);

  // ---- LDS DMA (inline asm: invisible to the compiler's vmcnt tracking). Instruction i (0, 1) of
  // wave w fills rows 16 i + 4 w + lane / 16 of a tile; the swizzle XOR terms depend on row & 15
  // (K) and row & 3 (V) only, the same for both i. Rows past S read as zeros (range check).
  const int prow = 4 * wave + (lane >> 4);
  const int kch = (lane & 15) ^ (prow & 15);
  const int vch = (lane & 15) ^ ((prow & 3) << 2);
  auto rsrc = [&](const unsigned short* base, int stride) __attribute__((always_inline)) {
    const unsigned long long a = (unsigned long long)(uintptr_t)(base + (size_t)b * S * stride + (size_t)hk * 128);
    return i32x4_t{__builtin_amdgcn_readfirstlane((int)(unsigned)a), __builtin_amdgcn_readfirstlane((int)(a >> 32)),
                   __builtin_amdgcn_readfirstlane(S * stride * 2), 0x00020000};
  };
  const i32x4_t rK = rsrc(K, k_stride), rV = rsrc(V, v_stride);
  const unsigned voffK = (unsigned)(prow * k_stride + kch * 8) * 2u;
  const unsigned voffV = (unsigned)(prow * v_stride + vch * 8) * 2u;
  const unsigned lds_base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const __amdgpu_buffer_rsrc_t bK = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(K + (size_t)b * S * k_stride + (size_t)hk * 128), (short)0, S * k_stride * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t bV = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(V + (size_t)b * S * v_stride + (size_t)hk * 128), (short)0, S * v_stride * 2, 0x00020000);
  auto dma = [&](const i32x4_t& r, unsigned voff, int stride, int t, unsigned lds) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int soff = __builtin_amdgcn_readfirstlane((t * W64_KT + 16 * i) * stride * 2);
      const unsigned dst = __builtin_amdgcn_readfirstlane(lds + i * 4096 + wave * 1024);
      if constexpr ((FLAGS & W64_BUILTIN_DMA) != 0) {   // diagnostics: the compiler's own LDS DMA
        __builtin_amdgcn_raw_ptr_buffer_load_lds(&r == &rK ? bK : bV,
                                                 (__attribute__((address_space(3))) void*)(uintptr_t)dst, 16, voff,
                                                 soff, 0, 0);
      } else {
        // one wait state between the M0 write and the DMA that reads it (hipcc emits the same
        // s_nop for its own LDS DMA; without it the DMA used the previous M0: tiles landed in
        // the wrong slot)
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :
                     : "s"(dst), "v"(voff), "s"(r), "s"(soff)
                     : "memory", "m0");
      }
    }
  };
  auto dma_tiles = [&](int j) __attribute__((always_inline)) {   // K(j+2), V(j) -> slot j & 1
    if (j + 2 < nkt) dma(rK, voffK, k_stride, j + 2, lds_base + (j & 1) * W64_TILE);
    if (j < nkt) dma(rV, voffV, v_stride, j, lds_base + 2 * W64_TILE + (j & 1) * W64_TILE);
  };
  auto sync = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((FLAGS & W64_T_NOBAR) == 0) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };

  // ---- fragments. K (A operand of QK^T) for d-step ds; V^T (A operand of P·V) for dim block dt,
  // 16-key step g (ds_read_b64_tr_b16 pair, as the ping-pong kernel). The swizzle makes the
  // per-lane part depend on ds (K) and dt (V) only: the key-step term is an immediate offset, so
  // 8 + 4 lane offsets serve every read of the loop.
  int kofs[8], vofs[4];
  {
    const int row = lane & 31, g16 = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) kofs[ds] = row * ROW8 + (k8swz(row, 2 * ds + hh) << 4);
    const int r0 = 8 * (g16 >> 1) + q4;                  // + 16 g; (r0 & 3) = q4 for every g
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) vofs[dt] = r0 * ROW8 + (v8swz(r0, 8 * dt + 4 * (g16 & 1) + p4) << 3);
  }
  auto kfrag = [&](const char* kb_, int ds) __attribute__((always_inline)) {
    return *(const bf16x8_t*)(kb_ + kofs[ds]);
  };
  auto vfrag = [&](const char* vb_, int dt, int g) __attribute__((always_inline)) {
    const char* a = vb_ + vofs[dt] + g * 16 * ROW8;
    const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a));
    const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a + 4 * ROW8));
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  // ---- softmax pieces on one S buffer -> the P buffer (per query block c)
  auto tile_max = [&](f32x16_t (&s)[2], int c) __attribute__((always_inline)) {
    float t = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) t = fmaxf(t, s[c][r]);
    return pair_max(t) * scale_log2;
  };
  // keys of tile j visible to row block c: register r is key j * 32 + 4 hh + (8 (r >> 2) + (r & 3));
  // rows see keys < lim (causal: their own position + 1). A tile no row of the wave may see
  // (past the diagonal, or past S) is masked whole, so its P is 0.
  auto mask = [&](f32x16_t (&s)[2], int j) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int qi = q0 + 32 * c + ql;
      const int rel = (causal ? min(qi + 1, S) : S) - (j * W64_KT + 4 * hh);
#pragma unroll
      for (int r = 0; r < 16; ++r) s[c][r] = (8 * (r >> 2) + (r & 3)) < rel ? s[c][r] : -INFINITY;
    }
  };
  auto exps = [&](f32x16_t (&s)[2], int c, int r0, float mneg) __attribute__((always_inline)) {
    float ps = 0.f;
#pragma unroll
    for (int r = r0; r < r0 + 8; ++r) {
      const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[c][r], scale_log2, mneg));
      s[c][r] = pv;
      ps += pv;
    }
    return ps;
  };
  auto pack = [&](f32x16_t (&s)[2], int c) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int rb = 8 * g;
      const unsigned lo0 = pack_bf16x2(s[c][rb + 0], s[c][rb + 1]);
      const unsigned lo1 = pack_bf16x2(s[c][rb + 2], s[c][rb + 3]);
      const unsigned hi0 = pack_bf16x2(s[c][rb + 4], s[c][rb + 5]);
      const unsigned hi1 = pack_bf16x2(s[c][rb + 6], s[c][rb + 7]);
      const auto w0 = __builtin_amdgcn_permlane32_swap(lo0, hi0, false, false);
      const auto w1 = __builtin_amdgcn_permlane32_swap(lo1, hi1, false, false);
      typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
      pP[c][g] = __builtin_bit_cast(bf16x8_t, u32x4_t{w0[0], w1[0], w0[1], w1[1]});
      asm volatile("" : "+a"(pP[c][g]));   // P waits for its P·V in AGPRs
    }
  };
  // online-softmax rescale of O, decided in step j (the row max grew by more than RESCALE_TAU:
  // rare, and once at the first tile, where O is still zero) and applied at the start of step
  // j + 1, after open()'s pad (every MFMA writing O has retired) and before P·V(j), the first
  // contribution at the new scale
  float pend_alpha[2] = {1.f, 1.f};
  bool pend = false;

  // ---- one step j: 32 MFMAs, each followed by its share of the step's other work (one work
  // slot per MFMA, fenced with sched_barrier so the compiler keeps the interleave): MFMAs 0-15
  // are P·V(j-1) (fragment fk = k >> 1: V^T of dims 32 (fk & 3) .., keys 16 (fk >> 2) ..; row
  // block c = k & 1), MFMAs 16-31 QK^T(j+1) (fragment fk = 8 + d-step; c = k & 1). Fragments
  // stream through a 3-deep ring, two fragments ahead. The work slots carry this step's DMA
  // (K(j+2), V(j)) and the softmax of tile j: row maxima, the rescale decision, 32 exponentials
  // two per slot, row sums, P packing. Branches (wave-uniform) only at the step's start —
  // before its first MFMA — and the step ends with a pad, so the allocator's copies at block
  // boundaries never read an unfinished MFMA.
  auto step = [&](int j, f32x16_t (&sc)[2], f32x16_t (&sn)[2]) __attribute__((always_inline)) {
    if (pend) {                 // one O tile at a time through VGPRs, back into its AGPRs
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          __builtin_amdgcn_sched_barrier(0);
          o[c][dt] *= pend_alpha[c];
          asm volatile("" : "+a"(o[c][dt]));
        }
      __builtin_amdgcn_sched_barrier(0);
      pend = false;
      asm volatile("s_nop 4" ::: "memory");        // VALU writes of O before the MFMAs read it
    }
    if (j >= mask_from) mask(sc, j);
    const char* vb = vbuf + ((j - 1) & 1) * W64_TILE;
    const char* kb_ = kbuf + ((j + 1) & 1) * W64_TILE;
    // this step's DMA is unconditional (no branch between MFMAs): a tile past S reads as zeros
    const unsigned lk = lds_base + (j & 1) * W64_TILE, lv = lds_base + 2 * W64_TILE + (j & 1) * W64_TILE;
    float t[2] = {-INFINITY, -INFINITY}, ps[2] = {0.f, 0.f};
    bf16x8_t ring[3];
    bf16x8_t (&qv)[2][8] = qf;   // named here: clang does not capture qf through the asm operands below
    auto load = [&](int fk) __attribute__((always_inline)) {
      ring[fk % 3] = fk < 8 ? vfrag(vb, fk & 3, fk >> 2) : kfrag(kb_, fk - 8);
    };
    auto mfma = [&](int k) __attribute__((always_inline)) {
      const int fk = k >> 1, c = k & 1;
      if (k < 16) {
        W64_MFMA_PV(o[c][fk & 3], ring[fk % 3], pP[c][fk >> 2]);
      } else if (fk == 8) {
        W64_MFMA_QK0(sn[c], ring[fk % 3], qv[c][0]);
      } else {
        W64_MFMA_QK(sn[c], ring[fk % 3], qv[c][fk - 8]);
      }
    };
    bf16x8_t stg[4];                           // W64_REGSTAGE: K rows (0, 1), V rows (2, 3) in flight
    auto dma1 = [&](const i32x4_t& r, unsigned voff, int stride, int tt, unsigned lds, int i) __attribute__((always_inline)) {
      const int soff = __builtin_amdgcn_readfirstlane((tt * W64_KT + 16 * i) * stride * 2);
      if constexpr ((FLAGS & W64_REGSTAGE) != 0) {
        // the load's destination is written when it lands: read only after the explicit vmcnt(0)
        asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=a"(stg[(&r == &rK ? 0 : 2) + i])
                     : "v"(voff), "s"(r), "s"(soff) : "memory");
      } else {
        const unsigned dst = __builtin_amdgcn_readfirstlane(lds + i * 4096 + wave * 1024);
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :
                     : "s"(dst), "v"(voff), "s"(r), "s"(soff)
                     : "memory", "m0");
      }
    };
    auto mx = [&](int c, int r0) __attribute__((always_inline)) {
#pragma unroll
      for (int r = r0; r < r0 + 8; ++r) t[c] = fmaxf(t[c], sc[c][r]);
    };
    auto ex = [&](int e) __attribute__((always_inline)) {      // 2 exponentials: row block e >> 3, regs 2 (e & 7) ..
      const int c = e >> 3, r = 2 * (e & 7);
#pragma unroll
      for (int i = 0; i < 2; ++i) sc[c][r + i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[c][r + i], scale_log2, -m[c]));
    };
    auto sm = [&](int c, int q) __attribute__((always_inline)) {   // row sum of regs 4 q .. 4 q + 3
#pragma unroll
      for (int r = 4 * q; r < 4 * q + 4; ++r) ps[c] += sc[c][r];
    };
    auto pk = [&](int c, int g) __attribute__((always_inline)) {
      const int rb = 8 * g;
      const unsigned lo0 = pack_bf16x2(sc[c][rb + 0], sc[c][rb + 1]);
      const unsigned lo1 = pack_bf16x2(sc[c][rb + 2], sc[c][rb + 3]);
      const unsigned hi0 = pack_bf16x2(sc[c][rb + 4], sc[c][rb + 5]);
      const unsigned hi1 = pack_bf16x2(sc[c][rb + 6], sc[c][rb + 7]);
      const auto w0 = __builtin_amdgcn_permlane32_swap(lo0, hi0, false, false);
      const auto w1 = __builtin_amdgcn_permlane32_swap(lo1, hi1, false, false);
      typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
      pP[c][g] = __builtin_bit_cast(bf16x8_t, u32x4_t{w0[0], w1[0], w0[1], w1[1]});
      asm volatile("" : "+a"(pP[c][g]));   // P waits for its P·V in AGPRs
    };
    auto work = [&](int k) __attribute__((always_inline)) {
      switch (k) {
        case 0: if constexpr ((FLAGS & W64_T_NODMA) == 0) dma1(rK, voffK, k_stride, j + 2, lk, 0); mx(0, 0); break;
        case 1: if constexpr ((FLAGS & W64_T_NODMA) == 0) dma1(rK, voffK, k_stride, j + 2, lk, 1); mx(0, 8); break;
        case 2: if constexpr ((FLAGS & W64_T_NODMA) == 0) dma1(rV, voffV, v_stride, j, lv, 0); mx(1, 0); break;
        case 3: if constexpr ((FLAGS & W64_T_NODMA) == 0) dma1(rV, voffV, v_stride, j, lv, 1); mx(1, 8); break;
        case 4:
          t[0] = pair_max(t[0]) * scale_log2;
          t[1] = pair_max(t[1]) * scale_log2;
          break;
        case 5: {
          const bool g0 = t[0] > m[0] + RESCALE_TAU, g1 = t[1] > m[1] + RESCALE_TAU;
          const float m0n = g0 ? t[0] : m[0], m1n = g1 ? t[1] : m[1];
          const float a0 = __builtin_amdgcn_exp2f(m[0] - m0n), a1 = __builtin_amdgcn_exp2f(m[1] - m1n);
          pend = __builtin_amdgcn_ballot_w64(g0 || g1) != 0;
          pend_alpha[0] = a0;
          pend_alpha[1] = a1;
          m[0] = m0n;
          m[1] = m1n;
          l[0] *= a0;
          l[1] *= a1;
          break;
        }
        case 22: sm(0, 0); sm(0, 1); break;
        case 23: sm(0, 2); sm(0, 3); break;
        case 24: sm(1, 0); sm(1, 1); break;
        case 25: sm(1, 2); sm(1, 3); break;
        case 26: pk(0, 0); break;
        case 27: pk(0, 1); break;
        case 28: pk(1, 0); break;
        case 29: pk(1, 1); break;
        case 30:
          l[0] += pair_sum(ps[0]);
          l[1] += pair_sum(ps[1]);
          break;
        default:
          if (k >= 6 && k < 22) ex(k - 6);
          break;
      }
    };
    load(0);
    load(1);
    // 32 slots, expanded at compile time (a rolled loop would index the fragment ring at run time)
    w64_static_for<0, 32>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      __builtin_amdgcn_sched_barrier(0);
      mfma(k);
      __builtin_amdgcn_sched_barrier(0);       // the slot's work stays behind its MFMA
      if constexpr ((k & 1) == 0 && (k >> 1) + 2 < 16) load((k >> 1) + 2);
      work(k);
    });
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((FLAGS & W64_PAD) != 0) asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
    if constexpr ((FLAGS & W64_REGSTAGE) != 0) {
      // the staged rows into this step's K / V slots (free since the barrier that opened the
      // step), at the lane-linear positions the DMA would have written
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned base = (i < 2 ? lk : lv) + (unsigned)((i & 1) * 4096 + wave * 1024 + lane * 16);
        asm volatile("ds_write_b128 %0, %1" ::"v"(base), "a"(stg[i]) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };

  // ---- prologue: zero P and the V ring (step 0's P·V(-1) then adds 0), K(0), K(1); S(0) = K(0) Q^T
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      pP[c][g] = bf16x8_t{};
      asm volatile("" : "+a"(pP[c][g]));
    }
#pragma unroll
  for (int i = 0; i < 2 * W64_TILE / (256 * 16); ++i)
    *(u16x8_t*)(vbuf + (i * 256 + tid) * 16) = u16x8_t{};
  if (0 < nkt) dma(rK, voffK, k_stride, 0, lds_base);
  if (1 < nkt) dma(rK, voffK, k_stride, 1, lds_base + W64_TILE);
  asm volatile("s_nop 4" ::: "memory");        // Q / P AGPR writes before their first MFMA read
  __syncthreads();                             // the V ring's zeros (LDS stores) before any read
  sync();
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) {
    const bf16x8_t f = kfrag(kbuf, ds);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      if (ds == 0)
        W64_MFMA_QK0(sA[c], f, qf[c][0]);
      else
        W64_MFMA_QK(sA[c], f, qf[c][ds]);
    }
  }
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");

  // ---- iterations j = 0, 1, ... (barriers and DMAs are collective: every wave runs the same
  // count, nkt + 1 rounded up to even): open() = wait for this wave's DMAs, barrier, DMA K(j+2)
  // and V(j) into the slots iteration j-1 finished reading. A wave computes steps j <= nlive
  // (step nlive is the last P·V; its softmax sees a fully masked tile and QK^T(nlive + 1) is
  // never used) and only stages tiles after that. S(j) is in sA for even j, sB for odd j.
  auto open = [&]() __attribute__((always_inline)) {
    sync();
    asm volatile("s_nop 2" ::: "memory");   // P's AGPR writes (last step) before the P·V MFMAs read them
  };
  // steps 0 .. nlive in pairs (no branch around a step inside the loop: a join there made the
  // allocator keep O in VGPRs and copy it into AGPRs every iteration), then the odd last step,
  // then staging-only iterations up to the block's common count
  int j = 0;
  for (; j + 1 <= nlive; j += 2) {
    open();
    step(j, sA, sB);
    open();
    step(j + 1, sB, sA);
  }
  if (j <= nlive) {
    open();
    step(j, sA, sB);
    ++j;
  }
  for (; j <= nkt; ++j) {            // every wave opens nkt + 1 iterations in all
    open();
    dma_tiles(j);
  }

  // ---- epilogue: O^T (AGPR) / l -> bf16 rows, widened stores
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int qi = q0 + 32 * c + ql;
    // O stays in AGPRs until here (pinned), so the loop's exit value is not copied to VGPRs early
    asm volatile("" : "+a"(o[c][0]), "+a"(o[c][1]), "+a"(o[c][2]), "+a"(o[c][3]));
    f32x16_t oc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) oc[dt] = o[c][dt];
    store_o_wide(oc, 1.f / l[c], O + (((size_t)b * S + min(qi, S - 1)) * Hq + h) * 128, hh, qi < S);
  }
}

template <int FLAGS = 0>
int launch_w64(const void* q, const void* k, const void* v, void* o, int B, int S, int Hq, int Hkv, int qs, int ks,
               int vs, float scale_log2, int causal, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)flash_fwd_d128_w64<FLAGS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              W64_LDS);
    attr = true;
  }
  const int nqb = (S + W64_QR - 1) / W64_QR;
  flash_fwd_d128_w64<FLAGS><<<dim3((unsigned)(B * Hq * nqb)), dim3(256), W64_LDS, stream>>>(
      (const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v, (unsigned short*)o, B, S, Hq,
      Hkv, qs, ks, vs, scale_log2, causal & 1);
  return gs_launch_status();
}

int g_attn_variant = 0;   // 0 = auto, 1 = 16x16 4-wave kernel, 2 = 32x32 4-wave, 3 = 32x32 8-wave

template <int NW, int FLAGS = 0>
int launch_w8(const void* q, const void* k, const void* v, void* o, int B, int S, int Hq, int Hkv, int qs, int ks,
              int vs, float scale_log2, int causal, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)flash_fwd_d128_w8<NW, FLAGS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS8);
    attr = true;
  }
  const int nqb = (S + 32 * NW - 1) / (32 * NW);
  flash_fwd_d128_w8<NW, FLAGS><<<dim3((unsigned)(B * Hq * nqb)), dim3(NW * 64), LDS8, stream>>>(
      (const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v, (unsigned short*)o, B, S, Hq,
      Hkv, qs, ks, vs, scale_log2, causal & 1);
  return gs_launch_status();
}

template <int D, bool TR>
int launch(const void* q, const void* k, const void* v, void* o, int B, int S, int Hq, int Hkv, int qs, int ks,
           int vs, float scale_log2, int causal, hipStream_t stream) {
  using C = Cfg<D>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)flash_fwd<D, TR>, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  const int nqb = (S + QROWS - 1) / QROWS;
  flash_fwd<D, TR><<<dim3((unsigned)(B * Hq * nqb)), dim3(256), C::LDS, stream>>>(
                     (const unsigned short*)q, (const unsigned short*)k, (const unsigned short*)v,
                     (unsigned short*)o, B, S, Hq, Hkv, qs, ks, vs, scale_log2, causal & 1);
  return gs_launch_status();
}

}  // namespace

// scale = softmax scale (1/sqrt(D) by default); strides are in elements between tokens.
GS_KERNEL_API int gs_flash_attn_fwd_bf16(const void* q, const void* k, const void* v, void* o, int B, int S, int Hq,
                                         int Hkv, int D, int q_stride, int k_stride, int v_stride, float scale,
                                         int causal, hipStream_t stream) {
  if (B <= 0 || S <= 0 || Hq <= 0 || Hkv <= 0 || Hq % Hkv || (D != 64 && D != 128) || q_stride < Hq * D ||
      k_stride < Hkv * D || v_stride < Hkv * D || q_stride % 8 || k_stride % 8 || v_stride % 8 ||
      ((uintptr_t)q & 15) || ((uintptr_t)k & 15) || ((uintptr_t)v & 15) || ((uintptr_t)o & 7))
    return GS_EINVAL;
  const float sl2 = scale * 1.4426950408889634f;
  // flags: bit0 causal, bit1 debug path (V^T fragments gathered without ds_read_b64_tr_b16)
  if (causal & 2)
    return D == 128 ? launch<128, false>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream)
                    : launch<64, false>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  // auto (measured on MI355X, tools/attn_sweep.py): the ping-pong 8-wave block wins on full
  // attention and causal S >= 2048 (1080-1110 / 1065-1095 TF/s at H 64 full / causal 8192 with the
  // widened store tail, profiles/r3/attn_sweep_wide_*.jsonl); on short causal sequences the
  // 4-wave block's finer granularity (128 rows, two blocks per CU) wins
  const bool pp_ok = (size_t)S * k_stride * 2 < (1ull << 31) && (size_t)S * v_stride * 2 < (1ull << 31);
  if (D == 128 && pp_ok && g_attn_variant == 8)
    return launch_pp<0>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 10)
    return launch_pp<PP_PRIO | PP_TRACE>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 12)
    return launch_pp<PP_SPRIO | PP_WIDE>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 14)
    return launch_w64<0>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 17)
    return launch_w64<W64_T_NOBAR>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 18)
    return launch_w64<W64_T_NODMA>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 19)
    return launch_w64<W64_T_NODMA | W64_T_NOBAR>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 20)
    return launch_w64<W64_REGSTAGE>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 16)
    return launch_w64<W64_PAD>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 15)
    return launch_w64<W64_BUILTIN_DMA>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && (g_attn_variant == 13 || g_attn_variant == 0))
    return launch_w8<4, AF_WIDE>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 9)
    return launch_pp<PP_PRIO | PP_ILV>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && g_attn_variant == 7)
    return launch_pp<PP_PRIO>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && pp_ok && (g_attn_variant == 11 || (g_attn_variant == 0 && (!(causal & 1) || S >= 2048))))
    return launch_pp<PP_PRIO | PP_WIDE>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && g_attn_variant == 4)
    return launch_w8<8, AF_PRIO>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && g_attn_variant == 5)
    return launch_w8<8, AF_LATE>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && g_attn_variant == 6)
    return launch_w8<4, AF_LATE>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  const bool w8 = g_attn_variant == 3;
  if (D == 128 && w8)
    return launch_w8<8>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  if (D == 128 && g_attn_variant != 1)
    return launch_w8<4>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
  return D == 128 ? launch<128, true>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream)
                  : launch<64, true>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
}

// Kernel selection for A/B measurement and tests: 0 = auto (32x32-MFMA kernels for D = 128:
// ping-pong 8-wave for full attention and causal S >= 2048, else 4-wave), 1 = the 16x16 4-wave kernel,
// 2 = 32x32 4-wave, 3 = 32x32 8-wave; experiments: 4 = 8-wave + younger-half priority, 5 = 8-wave
// + late (T14) loads, 6 = 4-wave + late loads, 7 = ping-pong 8-wave (MFMA-segment priority), 8 = ping-pong
// without the priority, 9 = ping-pong + interleaved partner rows (measured 1-3 % slower), 10 = ping-pong with the
// segment trace (gs_attn_trace), 11 = ping-pong + widened store tail, 12 = ping-pong with static
// younger-half priority + widened store tail, 13 = 4-wave 32x32 + widened store tail, 14 = one wave
// per SIMD with 64 rows (flash_fwd_d128_w64), 15 = the same with compiler-issued LDS DMA (diagnostics).
GS_KERNEL_API int gs_attn_set_variant(int v) {
  if (v < 0 || v > 20) return GS_EINVAL;
  g_attn_variant = v;
  return GS_OK;
}

// Segment trace of the last variant-10 launch: out[8 waves][PP_TRACE_SEGS][2] s_memtime stamps
// (0: before the barrier closing segment k, 1: after the barrier opening segment k).
GS_KERNEL_API int gs_attn_trace(unsigned long long* out, int n) {
  if (n < 8 * PP_TRACE_SEGS * 2) return GS_EINVAL;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pp_trace), sizeof(g_pp_trace)) == hipSuccess ? GS_OK : GS_EINVAL;
}
