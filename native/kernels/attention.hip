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
  const int bh = blockIdx.x / nqb;
  const int qb = causal ? (nqb - 1 - (int)(blockIdx.x % nqb)) : (int)(blockIdx.x % nqb);  // heaviest first
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
  return D == 128 ? launch<128, true>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream)
                  : launch<64, true>(q, k, v, o, B, S, Hq, Hkv, q_stride, k_stride, v_stride, sl2, causal, stream);
}
