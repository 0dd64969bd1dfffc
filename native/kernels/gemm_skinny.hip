// Skinny bf16 GEMM for decode: Y[M, N] = epilogue(X[M, K] · W[N, K]^T) with M <= 64 (the batch).
//
// In a decode step every projection reads its whole weight once for a handful of rows, so the
// kernel is an HBM stream over W. The large-tile GEMMs (gemm_bf16*.hip) would give the chip 16-112
// workgroups and waste 4-16x of their MFMA tile on padding rows. Schedule here:
//   * a wave owns 16 x NT output features (rows of W) over a K range; each lane streams 16-B
//     fragments of NT W rows (row = lane & 15 of each tile, k offset = (lane >> 4) * 8), 4 k-steps
//     of 32 in flight per batch of loads, and the activations X (<= 64 x K, L2-resident) come in
//     as the other MFMA operand (v_mfma_f32_16x16x32_bf16, MT = ceil(M / 16) row tiles), each
//     X fragment reused for the NT tiles;
//   * split-K so every shape launches >= ~2048 waves (8 per CU) to keep enough bytes in flight;
//     partial sums go to a float workspace [split, M, N] and a second kernel adds the splits,
//     the optional residual, and writes bf16. With one split the epilogue is fused instead.
// Accumulator layout (operands passed as (W, X)): lane holds Y[m = lane & 15][n0 + (lane >> 4) * 4 + r].
#include "common.h"

namespace {

constexpr int WAVES = 4;
constexpr int UNROLL = 4;             // k-steps of 32 loaded before their MFMAs

// A wave owns NT x 16 output features: every X fragment it loads feeds NT MFMAs, which divides the
// L2 -> CU traffic for X by NT (the first version, NT = 1, re-read X once per 16 features and was
// L2-bound at M >= 32: profiles/decode/README.md).
template <int MT, int NT>
__global__ __launch_bounds__(WAVES * 64) void skinny_nt(const unsigned short* __restrict__ X, int ldx,
                                                        const unsigned short* __restrict__ W, int ldw,
                                                        float* __restrict__ part, unsigned short* __restrict__ Y,
                                                        const unsigned short* __restrict__ R, int ldy, int M, int N,
                                                        int K, int kchunk) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * WAVES + wave) * 16 * NT;
  if (n0 >= N) return;
  const int split = blockIdx.y;
  const int k0 = split * kchunk, k1 = min(K, k0 + kchunk);
  const int r16 = lane & 15, kof = (lane >> 4) * 8;
  const unsigned short* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wp[j] = W + (size_t)(n0 + 16 * j + r16) * ldw + kof;
  const unsigned short* xp[MT];
  bool xok[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    xok[t] = t * 16 + r16 < M;
    xp[t] = X + (size_t)(xok[t] ? t * 16 + r16 : 0) * ldx + kof;
  }
  f32x4_t acc[MT][NT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[t][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // Register double buffer: the loads of k-block i + 1 are in flight while block i's MFMAs run
  // (the first version waited for every block's loads before its MFMAs: one exposed HBM latency
  // per block, with only ~2 waves per SIMD to cover it).
  bf16x8_t wa[UNROLL][NT], xa[UNROLL][MT], wb[UNROLL][NT], xb[UNROLL][MT];
  auto load = [&](bf16x8_t (&w)[UNROLL][NT], bf16x8_t (&x)[UNROLL][MT], int kk) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j) w[u][j] = *(const bf16x8_t*)(wp[j] + kk + 32 * u);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) x[u][t] = xok[t] ? *(const bf16x8_t*)(xp[t] + kk + 32 * u) : bf16x8_t{};
  };
  auto mma = [&](const bf16x8_t (&w)[UNROLL][NT], const bf16x8_t (&x)[UNROLL][MT]) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[u][j], x[u][t], acc[t][j], 0, 0, 0);
  };
  constexpr int STEP = 32 * UNROLL;
  int k = k0;
  if (k + 2 * STEP <= k1) {
    load(wa, xa, k);
    for (; k + 2 * STEP <= k1; k += 2 * STEP) {
      load(wb, xb, k + STEP);
      mma(wa, xa);
      if (k + 3 * STEP <= k1) load(wa, xa, k + 2 * STEP);
      mma(wb, xb);
    }
    if (k + STEP <= k1) {             // an odd block: its loads were issued by the last iteration
      mma(wa, xa);
      k += STEP;
    }
  }
  for (; k < k1; k += 32) {             // K tail in steps of 32 (K % 32 == 0 is required)
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const bf16x8_t x = xok[t] ? *(const bf16x8_t*)(xp[t] + k) : bf16x8_t{};
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8_t*)(wp[j] + k), x, acc[t][j], 0, 0, 0);
    }
  }

#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int nb = n0 + 16 * j + (lane >> 4) * 4;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = t * 16 + r16;
      if (m >= M) continue;
      if (part) {
        *(f32x4_t*)(part + ((size_t)split * M + m) * N + nb) = acc[t][j];
      } else {
        u16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[t][j][r];
          if (R) v += bf16_to_f32(R[(size_t)m * ldy + nb + r]);
          o[r] = f32_to_bf16(v);
        }
        *(u16x4_t*)(Y + (size_t)m * ldy + nb) = o;
      }
    }
  }
}

// LDS-staged variant: a workgroup owns 64 rows of W and stages 256-deep K slices of W and X in
// LDS, so every global load instruction reads 8 rows x 512 contiguous bytes (the register kernel
// above reads 16 rows x 64 B per instruction) and X is fetched once per workgroup instead of once
// per wave. The next slice's loads are in flight (in registers) while the MFMAs consume the
// current one. Rows are padded by 16 B in LDS to spread the 16-B fragment reads over the banks.
// NW = waves per workgroup (16 W rows each): 4; 2 (twice the workgroups) is selectable for
// measurement.
constexpr int LBN = 64, LBK = 256, LROW = LBK + 8;

// SWIGLU: W rows are gate/up interleaved by 16 (ops.interleave_gate_up), so even waves hold the
// gate and odd waves the up projection of the same 16 features; the unsplit epilogue writes
// Y[m, f] = silu(gate) * up (ldy = the F = N / 2 features) through LDS, and the separate
// SiLU·up kernel (one launch and a [M, N] round trip per layer) goes away.
// NORM: X is the residual stream h and the kernel stages rmsnorm(h) * nw instead: the producer's
// split reduction (skinny_reduce with ssq) left per-row partial sums of squares ssq[c][m] over
// nch chunks of the row, so inv_rms[m] = rsqrt(sum_c ssq / K + eps) is known up front and the
// scaling happens in the X staging pass (M x 256 values per k-slice): the RMSNorm kernel between
// the two projections (one launch per norm, 64 per decode step) goes away.
struct NormIn {
  const float* ssq;
  const unsigned short* w;
  int nch;
  float eps;
};

// PF = 2: two k-slices in flight per workgroup instead of one. A register ring of two slices
// (buffer loads; a slice past the workgroup's K range goes through a zero-size descriptor, so it
// costs no memory traffic and the load stream stays branch-free for the compiler's vmcnt
// accounting) — the next-but-one slice is requested before the current one is multiplied.
// PF = 3 (wave-level K split): every wave multiplies all 16 NW rows of the slice over its own
// quarter of the slice's K (LBK / NW) instead of its 16 rows over the whole slice, so each X
// fragment is read from LDS by one wave instead of all of them (per slice at M = 32: 48 instead
// of 96 KiB of fragment reads; M = 64: 64 instead of 160), and the NW partial tiles are summed
// through LDS once at the end; the epilogue then sees the usual tile-per-wave layout.
template <int MT, int NW, bool SWIGLU = false, bool NORM = false, int PF = 1>
__global__ __launch_bounds__(NW * 64) void skinny_lds(const unsigned short* __restrict__ X, int ldx,
                                                  const unsigned short* __restrict__ W, int ldw,
                                                  float* __restrict__ part, unsigned short* __restrict__ Y,
                                                  const unsigned short* __restrict__ R, int ldy, int M, int N, int K,
                                                  int kchunk, NormIn nrm = NormIn{}) {
  constexpr int RPI = 2 * NW;                             // rows per global load instruction
  // one LDS object (W image, then X image; reused for the wave-split reduction and the epilogue)
  __shared__ __attribute__((aligned(16))) unsigned short smem[(16 * NW + MT * 16) * LROW];
  unsigned short* const sW = smem;
  unsigned short* const sX = smem + 16 * NW * LROW;
  static_assert(PF != 3 || NW * NW * MT * 64 * 4 * 4 <= (16 * NW + MT * 16) * LROW * 2, "reduction fits LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16 * NW, split = blockIdx.y;
  const int k0 = split * kchunk, k1 = min(K, k0 + kchunk);
  if (k0 >= k1) return;
  const int lr = tid >> 5, lc = (tid & 31) * 8;           // global->LDS: row group, column
  constexpr int XI = MT * 16 / RPI;                       // X row groups (M padded to 16 MT)
  u16x8_t wr[8], xr[XI], nwr;
  float inv[XI];
  // NORM: up to 8 chunks (K <= 8192) of every row's sums of squares are loaded at once (clamped
  // addresses, masked adds in chunk order) before the first k-slice is requested, and summed after
  // it: one memory latency for both at the kernel's start instead of the sums' and then the slice's
  constexpr int NCH = 8;
  float cs[NORM ? XI : 1][NCH];
  if constexpr (NORM) {
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int m = min(RPI * i + lr, M - 1);
#pragma unroll
      for (int c = 0; c < NCH; ++c) cs[i][c] = nrm.ssq[(size_t)min(c, nrm.nch - 1) * M + m];
    }
  }
  auto norm_init = [&]() {
    if constexpr (NORM) {
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        const int m = RPI * i + lr;
        float ss = 0.f;
        if (nrm.nch <= NCH) {
#pragma unroll
          for (int c = 0; c < NCH; ++c) ss += c < nrm.nch ? cs[i][c] : 0.f;
        } else if (m < M) {
          for (int c = 0; c < nrm.nch; ++c) ss += nrm.ssq[(size_t)c * M + m];
        }
        inv[i] = rsqrtf(ss / (float)K + nrm.eps);
      }
    }
  };
  auto gload = [&](int kk) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const u16x8_t* src = (const u16x8_t*)(W + (size_t)(n0 + RPI * i + lr) * ldw + kk + lc);
      if constexpr (PF == 4)
        wr[i] = __builtin_nontemporal_load(src);     // streamed W: keep X resident in L2
      else
        wr[i] = *src;
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int m = RPI * i + lr;
      xr[i] = m < M ? *(const u16x8_t*)(X + (size_t)m * ldx + kk + lc) : u16x8_t{};
    }
    if constexpr (NORM) nwr = *(const u16x8_t*)(nrm.w + kk + lc);
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) *(u16x8_t*)(sW + (RPI * i + lr) * LROW + lc) = wr[i];
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      u16x8_t xv = xr[i];
      if constexpr (NORM) {
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] = f32_to_bf16(bf16_to_f32(xv[e]) * inv[i] * bf16_to_f32(nwr[e]));
      }
      *(u16x8_t*)(sX + (RPI * i + lr) * LROW + lc) = xv;
    }
  };
  f32x4_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, kof = (lane >> 4) * 8;
  const unsigned short* wl = sW + (16 * wave + r16) * LROW + kof;

  constexpr int KW = LBK / NW;                           // PF 3: k per wave per slice
  f32x4_t accw[PF == 3 ? NW : 1][MT];
  if constexpr (PF == 3) {
#pragma unroll
    for (int tt = 0; tt < NW; ++tt)
#pragma unroll
      for (int t = 0; t < MT; ++t) accw[tt][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  auto mma = [&]() {
    if constexpr (PF == 3) {
#pragma unroll
      for (int ks = 0; ks < KW / 32; ++ks) {
        const int kc = wave * KW + ks * 32 + kof;
        bf16x8_t xf[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) xf[t] = *(const bf16x8_t*)(sX + (16 * t + r16) * LROW + kc);
#pragma unroll
        for (int tt = 0; tt < NW; ++tt) {
          const bf16x8_t wf = *(const bf16x8_t*)(sW + (16 * tt + r16) * LROW + kc);
#pragma unroll
          for (int t = 0; t < MT; ++t)
            accw[tt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xf[t], accw[tt][t], 0, 0, 0);
        }
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < LBK / 32; ++ks) {
      const bf16x8_t wf = *(const bf16x8_t*)(wl + ks * 32);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const bf16x8_t xf = *(const bf16x8_t*)(sX + (16 * t + r16) * LROW + kof + ks * 32);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xf, acc[t], 0, 0, 0);
      }
    }
  };

  if constexpr (PF == 2) {
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    // descriptors: this workgroup's W rows, all of X (rows >= M read as zero), the norm weight
    const __amdgpu_buffer_rsrc_t rW =
        __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)n0 * ldw), (short)0, 16 * NW * ldw * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, M * ldx * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rN =
        __builtin_amdgcn_make_buffer_rsrc((void*)(NORM ? nrm.w : X), (short)0, NORM ? K * 2 : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, 0, 0x00020000);
    // the bounds check sees the VGPR offset only: rows go there, the k-slice into the SGPR offset
    const int vW = (lr * ldw + lc) * 2;
    u32x4_t w2[2][8], x2[2][XI], n2[2];
    auto gl = [&](u32x4_t(&wv)[8], u32x4_t(&xv)[XI], u32x4_t& nv, int kk) {
      const bool live = kk < k1;
      const __amdgpu_buffer_rsrc_t rw = live ? rW : rD, rx = live ? rX : rD, rn = live ? rN : rD;
#pragma unroll
      for (int i = 0; i < 8; ++i) wv[i] = __builtin_amdgcn_raw_buffer_load_b128(rw, vW, (RPI * i * ldw + kk) * 2, 0);
#pragma unroll
      for (int i = 0; i < XI; ++i)
        xv[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, ((RPI * i + lr) * ldx + lc) * 2, kk * 2, 0);
      if constexpr (NORM) nv = __builtin_amdgcn_raw_buffer_load_b128(rn, lc * 2, kk * 2, 0);
    };
    auto ls = [&](const u32x4_t(&wv)[8], const u32x4_t(&xv)[XI], const u32x4_t& nv) {
#pragma unroll
      for (int i = 0; i < 8; ++i) *(u32x4_t*)(sW + (RPI * i + lr) * LROW + lc) = wv[i];
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        u16x8_t xs = __builtin_bit_cast(u16x8_t, xv[i]);
        if constexpr (NORM) {
          const u16x8_t nw8 = __builtin_bit_cast(u16x8_t, nv);
#pragma unroll
          for (int e = 0; e < 8; ++e) xs[e] = f32_to_bf16(bf16_to_f32(xs[e]) * inv[i] * bf16_to_f32(nw8[e]));
        }
        *(u16x8_t*)(sX + (RPI * i + lr) * LROW + lc) = xs;
      }
    };
    // straight-line body (no mid-loop exit): every path into the loop head has exactly one
    // slice's loads (set 1) outstanding, so the compiler's vmcnt waits stay per-set
    const int S = (k1 - k0) / LBK;
    gl(w2[0], x2[0], n2[0], k0);
    gl(w2[1], x2[1], n2[1], k0 + LBK);
    norm_init();
    ls(w2[0], x2[0], n2[0]);
    __syncthreads();
    int it = 0;
    for (; it + 2 < S; it += 2) {                 // LDS: slice it; set 1: slice it + 1
      gl(w2[0], x2[0], n2[0], k0 + (it + 2) * LBK);
      mma();
      __syncthreads();
      ls(w2[1], x2[1], n2[1]);
      __syncthreads();
      gl(w2[1], x2[1], n2[1], k0 + (it + 3) * LBK);
      mma();
      __syncthreads();
      ls(w2[0], x2[0], n2[0]);
      __syncthreads();
    }
    mma();                                        // slice it (S - 2 or S - 1)
    if (it + 1 < S) {
      __syncthreads();
      ls(w2[1], x2[1], n2[1]);
      __syncthreads();
      mma();
    }
    __syncthreads();
  } else {                                       // PF 1 (and 4: the same with streamed W loads)
    gload(k0);
    norm_init();
    lstore();
    __syncthreads();
    for (int kk = k0; kk < k1; kk += LBK) {
      const bool more = kk + LBK < k1;
      if (more) gload(kk + LBK);
      mma();
      __syncthreads();
      if (more) {
        lstore();
        __syncthreads();
      }
    }
  }

  if constexpr (PF == 3) {
    // the last slice's barrier has passed: sum the NW waves' partial tiles, wave w gets tile w
    float* red = (float*)smem;                               // [wave][tile][MT][64 lanes] f32x4
#pragma unroll
    for (int tt = 0; tt < NW; ++tt)
#pragma unroll
      for (int t = 0; t < MT; ++t) *(f32x4_t*)(red + (((wave * NW + tt) * MT + t) * 64 + lane) * 4) = accw[tt][t];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      f32x4_t a = *(const f32x4_t*)(red + ((wave * MT + t) * 64 + lane) * 4);   // wave 0's tile `wave`
#pragma unroll
      for (int v = 1; v < NW; ++v) a += *(const f32x4_t*)(red + (((v * NW + wave) * MT + t) * 64 + lane) * 4);
      acc[t] = a;
    }
    __syncthreads();                                         // smem is the epilogue's again
  }
  const int nb = n0 + 16 * wave + (lane >> 4) * 4;
  if constexpr (SWIGLU) {
    // the last k-slice's barrier has passed: sW is free. Even waves park their gate tile there.
    float* gt = (float*)sW;                                // [NW / 2][MT * 16][16] floats
    const int pair = wave >> 1, c = (lane >> 4) * 4;
    if ((wave & 1) == 0) {
#pragma unroll
      for (int t = 0; t < MT; ++t) *(f32x4_t*)(gt + (pair * MT * 16 + t * 16 + r16) * 16 + c) = acc[t];
    }
    __syncthreads();
    if (wave & 1) {
      const int f = (n0 >> 1) + 16 * pair + c;             // output feature of this lane's 4 columns
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = t * 16 + r16;
        if (m >= M) continue;
        const f32x4_t g = *(const f32x4_t*)(gt + (pair * MT * 16 + t * 16 + r16) * 16 + c);
        u16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f32_to_bf16(g[r] / (1.f + __expf(-g[r])) * acc[t][r]);
        *(u16x4_t*)(Y + (size_t)m * ldy + f) = o;
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + r16;
    if (m >= M) continue;
    if (part) {
      *(f32x4_t*)(part + ((size_t)split * M + m) * N + nb) = acc[t];
    } else {
      u16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[t][r];
        if (R) v += bf16_to_f32(R[(size_t)m * ldy + nb + r]);
        o[r] = f32_to_bf16(v);
      }
      *(u16x4_t*)(Y + (size_t)m * ldy + nb) = o;
    }
  }
}

// Sum of the S split partials of 4 consecutive outputs at element offset i (stride MN between
// splits), added in split order. SPLITS > 0: a compile-time count, so all S loads are issued before
// the first add (one memory latency per thread instead of S in a row: the reductions are latency
// kernels, ~5 us each with the runtime loop); SPLITS = 0: the runtime count, in a loop.
template <int SPLITS>
__device__ __forceinline__ f32x4_t sum_splits(const float* __restrict__ part, int splits, size_t MN, size_t i) {
  if constexpr (SPLITS > 0) {
    f32x4_t v[SPLITS];
#pragma unroll
    for (int p = 0; p < SPLITS; ++p) v[p] = *(const f32x4_t*)(part + (size_t)p * MN + i);
    f32x4_t a = v[0];
#pragma unroll
    for (int p = 1; p < SPLITS; ++p) a += v[p];
    return a;
  } else {
    f32x4_t a = *(const f32x4_t*)(part + i);
    for (int p = 1; p < splits; ++p) a += *(const f32x4_t*)(part + (size_t)p * MN + i);
    return a;
  }
}

// Y[m, n] = sum_s part[s, m, n] (+ R[m, n]); 4 outputs per thread. With ssq (N % 1024 == 0) each
// 1024-element workgroup also writes the sum of squares of its stored bf16 outputs to
// ssq[chunk][m] (chunk = n / 1024): the next projection's RMSNorm, folded into its X staging.
template <int SPLITS>
__global__ __launch_bounds__(256) void skinny_reduce(const float* __restrict__ part, int splits,
                                                     unsigned short* __restrict__ Y, const unsigned short* __restrict__ R,
                                                     int ldy, int M, int N, float* __restrict__ ssq) {
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  float sq = 0.f;
  if (i < M * N) {
    const int m = i / N, n = i % N;
    const f32x4_t s = sum_splits<SPLITS>(part, splits, (size_t)M * N, i);
    u16x4_t o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = s[r];
      if (R) v += bf16_to_f32(R[(size_t)m * ldy + n + r]);
      o[r] = f32_to_bf16(v);
      const float q = bf16_to_f32(o[r]);
      sq += q * q;
    }
    *(u16x4_t*)(Y + (size_t)m * ldy + n) = o;
  }
  if (ssq) {
    __shared__ float red[4];
    sq = wave_sum(sq);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int e0 = blockIdx.x * 1024, m = e0 / N, c = (e0 % N) / 1024;
      ssq[(size_t)c * M + m] = red[0] + red[1] + red[2] + red[3];
    }
  }
}

// Decode fusion of the QKV projection's split reduction with RoPE(q), RoPE(k) and the KV-cache
// append (the rope_kv_append launch of decode_attention.hip goes away): per sequence b at
// position pos[b], the K splits of each rotation pair (d, d + 64) of a q / k head are summed,
// rounded to bf16 (as the reduction's stored output), rotated and written to Y, k also to the
// cache; v heads are summed, written to Y and appended raw. Y = [B, (Hq + 2 Hkv) * 128] rows.
struct RopeIn {
  const float* cosb;
  const float* sinb;
  int tab_rows;
  const int* pos;
  unsigned short* kc;
  unsigned short* vc;
  int hq, hkv, smax;
};

template <int SPLITS>
__global__ __launch_bounds__(256) void skinny_reduce_rope(const float* __restrict__ part, int splits,
                                                          unsigned short* __restrict__ Y, int ldy, int M, int N,
                                                          RopeIn rp) {
  constexpr int D = 128, HALF = D / 2, NQ = HALF / 4, NV = D / 8;
  const int per = (rp.hq + rp.hkv) * NQ + rp.hkv * NV;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * per) return;
  const int b = i / per, r = i % per;
  const int p = rp.pos[b];
  const bool in_cache = p >= 0 && p < rp.smax;
  auto sum4 = [&](int n) { return sum_splits<SPLITS>(part, splits, (size_t)M * N, (size_t)b * N + n); };
  unsigned short* row = Y + (size_t)b * ldy;
  if (r < (rp.hq + rp.hkv) * NQ) {
    const int h = r / NQ, d = (r % NQ) * 4, n = h * D + d;
    const f32x4_t a = sum4(n), c2 = sum4(n + HALF);
    const int pt = min(max(p, 0), rp.tab_rows - 1);
    const float4 c = *(const float4*)(rp.cosb + (size_t)pt * HALF + d);
    const float4 sn = *(const float4*)(rp.sinb + (size_t)pt * HALF + d);
    const float cc[4] = {c.x, c.y, c.z, c.w}, sc[4] = {sn.x, sn.y, sn.z, sn.w};
    u16x4_t oa, ob;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x1 = bf16_to_f32(f32_to_bf16(a[e])), x2 = bf16_to_f32(f32_to_bf16(c2[e]));
      oa[e] = f32_to_bf16(x1 * cc[e] - x2 * sc[e]);
      ob[e] = f32_to_bf16(x2 * cc[e] + x1 * sc[e]);
    }
    *(u16x4_t*)(row + n) = oa;
    *(u16x4_t*)(row + n + HALF) = ob;
    if (h >= rp.hq && in_cache) {
      unsigned short* dst = rp.kc + ((((size_t)b * rp.hkv + (h - rp.hq)) * rp.smax + p) * D);
      *(u16x4_t*)(dst + d) = oa;
      *(u16x4_t*)(dst + HALF + d) = ob;
    }
  } else {
    const int r2 = r - (rp.hq + rp.hkv) * NQ, h = r2 / NV, c = (r2 % NV) * 8;
    const int n = (rp.hq + rp.hkv + h) * D + c;
    const f32x4_t lo = sum4(n), hi = sum4(n + 4);
    u16x8_t o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = f32_to_bf16(lo[e]);
      o[e + 4] = f32_to_bf16(hi[e]);
    }
    *(u16x8_t*)(row + n) = o;
    if (in_cache) *(u16x8_t*)(rp.vc + ((((size_t)b * rp.hkv + h) * rp.smax + p) * D) + c) = o;
  }
}

// Decode fusion of the split reduction with the RMSNorm that always follows a residual
// projection: per row m, h = sum_s part[s, m, :] + R[m, :] (or h = Y[m, :] when the GEMM ran
// unsplit and already wrote it), Y = bf16(h), xn = bf16(h * rsqrt(mean(h^2) + eps) * nw) with
// the norm taken over the stored bf16 values, as ops.rmsnorm does. One workgroup per row.
__global__ __launch_bounds__(256) void skinny_reduce_norm(const float* __restrict__ part, int splits,
                                                          unsigned short* __restrict__ Y,
                                                          const unsigned short* __restrict__ R, int ldy, int M, int N,
                                                          const unsigned short* __restrict__ nw,
                                                          unsigned short* __restrict__ xn, int ldxn, float eps) {
  constexpr int MAXV = 4;                       // N <= 256 threads x 4 vectors x 8 = 8192
  const int m = blockIdx.x, nvec = N / 8;
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int t = 0; t < MAXV; ++t) {
    const int vi = threadIdx.x + t * 256;
    if (vi >= nvec) continue;
    const int n = vi * 8;
    u16x8_t hv;
    if (part) {
      f32x4_t a = *(const f32x4_t*)(part + (size_t)m * N + n), b = *(const f32x4_t*)(part + (size_t)m * N + n + 4);
      for (int p = 1; p < splits; ++p) {
        a += *(const f32x4_t*)(part + ((size_t)p * M + m) * N + n);
        b += *(const f32x4_t*)(part + ((size_t)p * M + m) * N + n + 4);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float h = e < 4 ? a[e] : b[e - 4];
        if (R) h += bf16_to_f32(R[(size_t)m * ldy + n + e]);
        hv[e] = f32_to_bf16(h);
      }
      *(u16x8_t*)(Y + (size_t)m * ldy + n) = hv;
    } else {
      hv = *(const u16x8_t*)(Y + (size_t)m * ldy + n);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[t][e] = bf16_to_f32(hv[e]);
      ss += v[t][e] * v[t][e];
    }
  }
  __shared__ float red[4];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float inv = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)N + eps);
#pragma unroll
  for (int t = 0; t < MAXV; ++t) {
    const int vi = threadIdx.x + t * 256;
    if (vi >= nvec) continue;
    const u16x8_t wv = *(const u16x8_t*)(nw + vi * 8);
    u16x8_t o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(v[t][e] * inv * bf16_to_f32(wv[e]));
    *(u16x8_t*)(xn + (size_t)m * ldxn + vi * 8) = o;
  }
}

}  // namespace

// Features per wave (16 x NT) and split-K factor for a shape: NT = 4 once the grid has >= 1024
// such waves, else 2, else 1; then splits double (keeping >= 256 k per split) until ~2048 waves.
static int g_force_nt = 0;   // 0 = heuristic; 1 / 2 / 4 = forced (sweeps, tests)
static int g_variant = 0;    // 0 = auto (LDS-staged when K % 256 == 0), 1 = register kernel, 2 = LDS

static bool use_lds(int K) { return g_variant == 2 || (g_variant == 0 && K % LBK == 0); }

static int g_lds_waves = 0;  // 0 = default (4); 2 / 4 forced
// 4-wave LDS schedule: 0 = auto, 1 = one k-slice in flight, 2 = two, 3 = wave-level K split,
// 4 = one slice with W loaded non-temporal. Auto streams W non-temporal when it is >= 64 MiB and
// loads it plainly otherwise. Measured with weights streamed from HBM, as in a decode step
// (profiles/decode/skinny_nt_r3_micro.jsonl): nt keeps the W stream from evicting X in L2 and runs
// the gate/up, down and LM-head projections 4-9 % faster; the 34-50 MB qkv / o weights lose 0-8 %.
static int g_pf = 0;

GS_KERNEL_API int gs_skinny_set_prefetch(int pf) {
  if (pf < 0 || pf > 4) return GS_EINVAL;
  g_pf = pf;
  return GS_OK;
}

GS_KERNEL_API int gs_skinny_get_prefetch() { return g_pf; }

// Launch the 4-wave LDS kernel <MT, SWIGLU, NORM> with the schedule g_pf selects.
template <int MT, bool SWIGLU, bool NORM, typename Go>
static void go_lds4(Go&& go, size_t wbytes) {
  switch (g_pf ? g_pf : wbytes >= (64u << 20) ? 4 : 1) {
    case 2: go(skinny_lds<MT, 4, SWIGLU, NORM, 2>); break;
    case 3: go(skinny_lds<MT, 4, SWIGLU, NORM, 3>); break;
    case 4: go(skinny_lds<MT, 4, SWIGLU, NORM, 4>); break;
    default: go(skinny_lds<MT, 4, SWIGLU, NORM, 1>); break;
  }
}

// 2-wave workgroups were measured slower on every decode shape (each workgroup re-stages X, and
// the gate/up went 39 -> 46 us at batch 32: profiles/decode/micro_lds_waves.jsonl), so 4 it is.
static int lds_waves(int) { return g_lds_waves ? g_lds_waves : 4; }

GS_KERNEL_API int gs_skinny_set_lds_waves(int nw) {
  if (nw != 0 && nw != 2 && nw != 4) return GS_EINVAL;
  g_lds_waves = nw;
  return GS_OK;
}

// LDS variant: 64 features per workgroup; splits double (>= 512 k each) until the grid has
// g_wg_target workgroups, unless W is wide enough (>= 256 workgroups) on its own. Measured on
// MI355X over targets 256-2048 (profiles/decode/micro_lds_wg_sweep.jsonl): splitting the 28672-wide
// gate/up projection cost 10-20 %, splitting the 4096-wide ones to 512 workgroups won 10-25 %.
static int g_wg_target = 512;

static void plan_lds(int N, int K, int& splits) {
  splits = 1;
  if (N / LBN >= 256) return;   // wide W: the split partials cost more than the parallelism gains
  while ((N / LBN) * splits < g_wg_target && K / (splits * 2) >= 512) splits *= 2;
}

GS_KERNEL_API int gs_skinny_set_wg_target(int n) {
  if (n < 1 || n > 65536) return GS_EINVAL;
  g_wg_target = n;
  return GS_OK;
}

static void plan(int N, int K, int& nt, int& splits) {
  nt = g_force_nt ? g_force_nt : N / 64 >= 1024 ? 4 : N / 32 >= 512 ? 2 : 1;
  const int waves = N / (16 * nt);
  splits = 1;
  while (waves * splits < 2048 && K / (splits * 2) >= 256) splits *= 2;
}

GS_KERNEL_API int gs_skinny_set_nt(int nt) {
  if (nt != 0 && nt != 1 && nt != 2 && nt != 4) return GS_EINVAL;
  g_force_nt = nt;
  return GS_OK;
}

GS_KERNEL_API int gs_skinny_set_variant(int v) {
  if (v < 0 || v > 2) return GS_EINVAL;
  g_variant = v;
  return GS_OK;
}

GS_KERNEL_API int gs_skinny_splits(int N, int K) {
  int nt, s;
  if (use_lds(K)) {
    plan_lds(N, K, s);
    return s;
  }
  plan(N, K, nt, s);
  return s;
}

// X [M, K] (ldx), W [N, K] (ldw), Y [M, N] (ldy), optional residual R with Y's layout (may alias Y).
// part: float workspace of splits * M * N (ignored when splits == 1). Requires M in [1, 64],
// N % 64 == 0, K % 32 == 0, ldx / ldw % 8 == 0, ldy % 4 == 0, 16-B aligned X and W.
// Post-GEMM step: the plain split reduction, or (nw != null) the reduction fused with RMSNorm.
static int g_reduce_static = 1;   // split reductions with compile-time split counts (0: runtime loop, A/B)

GS_KERNEL_API int gs_skinny_set_reduce_static(int on) {
  if (on != 0 && on != 1) return GS_EINVAL;
  g_reduce_static = on;
  return GS_OK;
}

static thread_local float* g_ssq_out = nullptr;   // skinny_reduce writes row sums of squares here
static thread_local NormIn g_norm_in{};            // skinny_lds stages rmsnorm(X) when g_norm_in.ssq is set
static thread_local RopeIn g_rope_in{};            // split reduction = skinny_reduce_rope when g_rope_in.pos is set

static void finish(float* pp, int nsplit, void* Y, const void* R, int ldy, int M, int N, const void* nw, void* xn,
                   int ldxn, float eps, hipStream_t stream) {
  if (g_rope_in.pos) {
    const int n = M * ((g_rope_in.hq + g_rope_in.hkv) * 16 + g_rope_in.hkv * 16);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((n + 255) / 256), dim3(256), 0, stream, (const float*)pp, nsplit,
                         (unsigned short*)Y, ldy, M, N, g_rope_in);
    };
    switch (g_reduce_static ? nsplit : 0) {
      case 2: go(skinny_reduce_rope<2>); break;
      case 4: go(skinny_reduce_rope<4>); break;
      case 8: go(skinny_reduce_rope<8>); break;
      case 16: go(skinny_reduce_rope<16>); break;
      default: go(skinny_reduce_rope<0>); break;
    }
  } else if (nw) {
    hipLaunchKernelGGL(skinny_reduce_norm, dim3(M), dim3(256), 0, stream, (const float*)pp, nsplit,
                       (unsigned short*)Y, (const unsigned short*)R, ldy, M, N, (const unsigned short*)nw,
                       (unsigned short*)xn, ldxn, eps);
  } else if (pp) {
    const int n4 = M * N / 4;
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((n4 + 255) / 256), dim3(256), 0, stream, (const float*)pp, nsplit,
                         (unsigned short*)Y, (const unsigned short*)R, ldy, M, N, g_ssq_out);
    };
    switch (g_reduce_static ? nsplit : 0) {
      case 2: go(skinny_reduce<2>); break;
      case 4: go(skinny_reduce<4>); break;
      case 8: go(skinny_reduce<8>); break;
      case 16: go(skinny_reduce<16>); break;
      default: go(skinny_reduce<0>); break;
    }
  }
}

static int skinny_launch(const void* X, int ldx, const void* W, int ldw, void* Y, const void* R, int ldy, int M, int N,
                         int K, int splits, void* part, const void* nw, void* xn, int ldxn, float eps,
                         hipStream_t stream) {
  if (M < 1 || M > 64 || N % 64 || K % 32 || K <= 0 || ldx % 8 || ldw % 8 || ldy % 4 || ldx < K || ldw < K ||
      ldy < N || splits < 1 || (splits > 1 && !part))
    return GS_EINVAL;
  const int mt = (M + 15) / 16;
  if (use_lds(K)) {
    if (K % LBK) return GS_EINVAL;
    int kchunk = (K + splits - 1) / splits;
    kchunk = (kchunk + LBK - 1) / LBK * LBK;
    const int nsplit = (K + kchunk - 1) / kchunk;
    float* pp = nsplit > 1 ? (float*)part : nullptr;
    // the RoPE / KV-append epilogue lives in the split reduction: split, no residual, QKV width
    if (g_rope_in.pos && (!pp || R || nw || ldy % 8 || N != (g_rope_in.hq + 2 * g_rope_in.hkv) * 128))
      return GS_EINVAL;
    const int waves = lds_waves(N);
    const dim3 grid(N / (16 * waves), nsplit);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, grid, dim3(waves * 64), 0, stream, (const unsigned short*)X, ldx, (const unsigned short*)W,
                         ldw, pp, (unsigned short*)Y, (const unsigned short*)R, ldy, M, N, K, kchunk, g_norm_in);
    };
    if (g_norm_in.ssq) {
      if (waves != 4) return GS_EINVAL;
      switch (mt) {
        case 1: go_lds4<1, false, true>(go, (size_t)N * K * 2); break;
        case 2: go_lds4<2, false, true>(go, (size_t)N * K * 2); break;
        case 3: go_lds4<3, false, true>(go, (size_t)N * K * 2); break;
        default: go_lds4<4, false, true>(go, (size_t)N * K * 2); break;
      }
      finish(pp, nsplit, Y, R, ldy, M, N, nw, xn, ldxn, eps, stream);
      return gs_launch_status();
    }
    switch (mt) {
      case 1: waves == 2 ? go(skinny_lds<1, 2>) : go_lds4<1, false, false>(go, (size_t)N * K * 2); break;
      case 2: waves == 2 ? go(skinny_lds<2, 2>) : go_lds4<2, false, false>(go, (size_t)N * K * 2); break;
      case 3: waves == 2 ? go(skinny_lds<3, 2>) : go_lds4<3, false, false>(go, (size_t)N * K * 2); break;
      default: waves == 2 ? go(skinny_lds<4, 2>) : go_lds4<4, false, false>(go, (size_t)N * K * 2); break;
    }
    finish(pp, nsplit, Y, R, ldy, M, N, nw, xn, ldxn, eps, stream);
    return gs_launch_status();
  }
  if (g_norm_in.ssq || g_rope_in.pos) return GS_EINVAL;   // folded norm / RoPE epilogue: LDS kernel only
  int nt, planned;
  plan(N, K, nt, planned);
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + 255) / 256 * 256;
  const int nsplit = (K + kchunk - 1) / kchunk;
  float* pp = nsplit > 1 ? (float*)part : nullptr;
  const int per_wg = 16 * nt * WAVES;
  const dim3 grid((N + per_wg - 1) / per_wg, nsplit);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(WAVES * 64), 0, stream, (const unsigned short*)X, ldx,
                       (const unsigned short*)W, ldw, pp, (unsigned short*)Y, (const unsigned short*)R, ldy, M, N, K,
                       kchunk);
  };
#define GS_SKINNY_NT(NT_)                     \
  switch (mt) {                               \
    case 1: go(skinny_nt<1, NT_>); break;     \
    case 2: go(skinny_nt<2, NT_>); break;     \
    case 3: go(skinny_nt<3, NT_>); break;     \
    default: go(skinny_nt<4, NT_>); break;    \
  }
  if (nt == 4) {
    GS_SKINNY_NT(4)
  } else if (nt == 2) {
    GS_SKINNY_NT(2)
  } else {
    GS_SKINNY_NT(1)
  }
#undef GS_SKINNY_NT
  finish(pp, nsplit, Y, R, ldy, M, N, nw, xn, ldxn, eps, stream);
  return gs_launch_status();
}

GS_KERNEL_API int gs_skinny_gemm_bf16(const void* X, int ldx, const void* W, int ldw, void* Y, const void* R, int ldy,
                                      int M, int N, int K, int splits, void* part, hipStream_t stream) {
  return skinny_launch(X, ldx, W, ldw, Y, R, ldy, M, N, K, splits, part, nullptr, nullptr, 0, 0.f, stream);
}

// Same GEMM, then xn = RMSNorm(Y) * nw in the reduction pass (N % 8 == 0, N <= 8192, ldxn % 8 == 0).
GS_KERNEL_API int gs_skinny_gemm_norm_bf16(const void* X, int ldx, const void* W, int ldw, void* Y, const void* R,
                                           int ldy, int M, int N, int K, int splits, void* part, const void* nw,
                                           void* xn, int ldxn, float eps, hipStream_t stream) {
  if (!nw || !xn || N > 8192 || ldy % 8 || ldxn % 8 || ldxn < N) return GS_EINVAL;
  return skinny_launch(X, ldx, W, ldw, Y, R, ldy, M, N, K, splits, part, nw, xn, ldxn, eps, stream);
}

// Y[M, F] = silu(X W_gate^T) * (X W_up^T) for W [2F, K] gate/up interleaved by 16 rows
// (ops.interleave_gate_up): one launch, LDS kernel, unsplit (W wide enough: 2F / 64 >= 256
// workgroups, i.e. F >= 8192; narrower shapes return GS_EINVAL and the caller runs GEMM + SiLU·up).
GS_KERNEL_API int gs_skinny_swiglu_bf16(const void* X, int ldx, const void* W, int ldw, void* Y, int ldy, int M,
                                        int F, int K, hipStream_t stream) {
  const int N = 2 * F;
  int splits;
  if (g_rope_in.pos || M < 1 || M > 64 || F % 32 || K % LBK || K <= 0 || ldx % 8 || ldw % 8 || ldy % 4 || ldx < K || ldw < K ||
      ldy < F || !use_lds(K) || lds_waves(N) != 4)
    return GS_EINVAL;
  plan_lds(N, K, splits);
  if (splits != 1) return GS_EINVAL;
  const dim3 grid(N / 64, 1);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, (const unsigned short*)X, ldx, (const unsigned short*)W, ldw,
                       (float*)nullptr, (unsigned short*)Y, (const unsigned short*)nullptr, ldy, M, N, K, K, g_norm_in);
  };
  if (g_norm_in.ssq) {
    switch ((M + 15) / 16) {
      case 1: go_lds4<1, true, true>(go, (size_t)N * K * 2); break;
      case 2: go_lds4<2, true, true>(go, (size_t)N * K * 2); break;
      case 3: go_lds4<3, true, true>(go, (size_t)N * K * 2); break;
      default: go_lds4<4, true, true>(go, (size_t)N * K * 2); break;
    }
  } else {
    switch ((M + 15) / 16) {
      case 1: go_lds4<1, true, false>(go, (size_t)N * K * 2); break;
      case 2: go_lds4<2, true, false>(go, (size_t)N * K * 2); break;
      case 3: go_lds4<3, true, false>(go, (size_t)N * K * 2); break;
      default: go_lds4<4, true, false>(go, (size_t)N * K * 2); break;
    }
  }
  return gs_launch_status();
}

// Per-launch options of the next skinny call on this thread of the host: ssq_out (float
// [N / 1024][M]) makes the split reduction emit row sums of squares (requires a split GEMM and
// N % 1024 == 0); norm_ssq / norm_w / nch / eps make the GEMM stage rmsnorm(X) * norm_w of its
// X rows. Both reset to off by gs_skinny_clear_opts (the Python wrapper brackets each call).
GS_KERNEL_API int gs_skinny_set_opts(float* ssq_out, const float* norm_ssq, const void* norm_w, int nch, float eps) {
  if ((norm_ssq == nullptr) != (norm_w == nullptr) || (norm_ssq && nch <= 0)) return GS_EINVAL;
  g_ssq_out = ssq_out;
  g_norm_in = NormIn{norm_ssq, (const unsigned short*)norm_w, nch, eps};
  return GS_OK;
}

GS_KERNEL_API int gs_skinny_clear_opts() {
  g_ssq_out = nullptr;
  g_norm_in = NormIn{};
  g_rope_in = RopeIn{};
  return GS_OK;
}

// Per-launch option: the next skinny call's split reduction applies RoPE(q, k) at pos[b] and
// appends k / v to the caches [B, Hkv, Smax, 128] (skinny_reduce_rope); the call returns
// GS_EINVAL unless it splits, has no residual and N = (Hq + 2 Hkv) * 128. Cleared with the rest.
GS_KERNEL_API int gs_skinny_set_rope(const float* cosb, const float* sinb, int tab_rows, const int* pos, void* kc,
                                     void* vc, int hq, int hkv, int smax) {
  if (!cosb || !sinb || !pos || !kc || !vc || tab_rows <= 0 || hq <= 0 || hkv <= 0 || smax <= 0) return GS_EINVAL;
  g_rope_in = RopeIn{cosb, sinb, tab_rows, pos, (unsigned short*)kc, (unsigned short*)vc, hq, hkv, smax};
  return GS_OK;
}

