// Skinny bf16 GEMM for decode: Y[M, N] = epilogue(X[M, K] · W[N, K]^T) with M <= 64 (the batch).
//
// In a decode step every projection reads its whole weight once for a handful of rows, so the
// kernel is an HBM stream over W. The large-tile GEMMs (gemm_bf16*.hip) would give the chip 16-112
// workgroups and waste 4-16x of their MFMA tile on padding rows. Schedule here:
//   * a wave owns 16 output features (16 rows of W) over a K range; each lane streams 16-B
//     fragments of one W row (row = lane & 15, k offset = (lane >> 4) * 8), 8 MFMA steps of
//     k = 32 in flight per batch of loads, and the activations X (<= 64 x K, L2-resident) come in
//     as the other MFMA operand (v_mfma_f32_16x16x32_bf16, MT = ceil(M / 16) row tiles);
//   * split-K so every shape launches >= ~2048 waves (8 per CU) to keep enough bytes in flight;
//     partial sums go to a float workspace [split, M, N] and a second kernel adds the splits,
//     the optional residual, and writes bf16. With one split the epilogue is fused instead.
// Accumulator layout (operands passed as (W, X)): lane holds Y[m = lane & 15][n0 + (lane >> 4) * 4 + r].
#include "common.h"

namespace {

constexpr int WAVES = 4;
constexpr int UNROLL = 8;             // k-steps of 32 loaded before their MFMAs (8 x 16 B per lane in flight)

template <int MT>
__global__ __launch_bounds__(WAVES * 64) void skinny_nt(const unsigned short* __restrict__ X, int ldx,
                                                        const unsigned short* __restrict__ W, int ldw,
                                                        float* __restrict__ part, unsigned short* __restrict__ Y,
                                                        const unsigned short* __restrict__ R, int ldy, int M, int N,
                                                        int K, int kchunk) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * WAVES + wave) * 16;
  if (n0 >= N) return;
  const int split = blockIdx.y;
  const int k0 = split * kchunk, k1 = min(K, k0 + kchunk);
  const int r16 = lane & 15, kof = (lane >> 4) * 8;
  const unsigned short* wp = W + (size_t)(n0 + r16) * ldw + kof;
  const unsigned short* xp[MT];
  bool xok[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    xok[t] = t * 16 + r16 < M;
    xp[t] = X + (size_t)(xok[t] ? t * 16 + r16 : 0) * ldx + kof;
  }
  f32x4_t acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  int k = k0;
  for (; k + 32 * UNROLL <= k1; k += 32 * UNROLL) {
    bf16x8_t w[UNROLL], x[UNROLL][MT];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) w[u] = *(const bf16x8_t*)(wp + k + 32 * u);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t)
        x[u][t] = xok[t] ? *(const bf16x8_t*)(xp[t] + k + 32 * u) : bf16x8_t{};
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[u], x[u][t], acc[t], 0, 0, 0);
  }
  for (; k < k1; k += 32) {             // K tail in steps of 32 (K % 32 == 0 is required)
    const bf16x8_t w = *(const bf16x8_t*)(wp + k);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const bf16x8_t x = xok[t] ? *(const bf16x8_t*)(xp[t] + k) : bf16x8_t{};
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x, acc[t], 0, 0, 0);
    }
  }

  const int nb = n0 + (lane >> 4) * 4;
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

// Y[m, n] = sum_s part[s, m, n] (+ R[m, n]); 4 outputs per thread.
__global__ __launch_bounds__(256) void skinny_reduce(const float* __restrict__ part, int splits,
                                                     unsigned short* __restrict__ Y, const unsigned short* __restrict__ R,
                                                     int ldy, int M, int N) {
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= M * N) return;
  const int m = i / N, n = i % N;
  f32x4_t s = *(const f32x4_t*)(part + i);
  for (int p = 1; p < splits; ++p) s += *(const f32x4_t*)(part + (size_t)p * M * N + i);
  u16x4_t o;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = s[r];
    if (R) v += bf16_to_f32(R[(size_t)m * ldy + n + r]);
    o[r] = f32_to_bf16(v);
  }
  *(u16x4_t*)(Y + (size_t)m * ldy + n) = o;
}

}  // namespace

// Splits chosen so the grid has >= 2048 waves (or K runs out); kchunk a multiple of 256.
GS_KERNEL_API int gs_skinny_splits(int N, int K) {
  const int waves = N / 16;
  int s = 1;
  while (waves * s < 2048 && K / (s * 2) >= 512) s *= 2;
  return s;
}

// X [M, K] (ldx), W [N, K] (ldw), Y [M, N] (ldy), optional residual R with Y's layout (may alias Y).
// part: float workspace of splits * M * N (ignored when splits == 1). Requires M in [1, 64],
// N % 64 == 0, K % 32 == 0, ldx / ldw % 8 == 0, ldy % 4 == 0, 16-B aligned X and W.
GS_KERNEL_API int gs_skinny_gemm_bf16(const void* X, int ldx, const void* W, int ldw, void* Y, const void* R, int ldy,
                                      int M, int N, int K, int splits, void* part, hipStream_t stream) {
  if (M < 1 || M > 64 || N % 64 || K % 32 || K <= 0 || ldx % 8 || ldw % 8 || ldy % 4 || ldx < K || ldw < K ||
      ldy < N || splits < 1 || (splits > 1 && !part))
    return GS_EINVAL;
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + 255) / 256 * 256;
  const int nsplit = (K + kchunk - 1) / kchunk;
  float* pp = nsplit > 1 ? (float*)part : nullptr;
  const dim3 grid(N / (16 * WAVES), nsplit);
  const int mt = (M + 15) / 16;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(WAVES * 64), 0, stream, (const unsigned short*)X, ldx,
                       (const unsigned short*)W, ldw, pp, (unsigned short*)Y, (const unsigned short*)R, ldy, M, N, K,
                       kchunk);
  };
  switch (mt) {
    case 1: go(skinny_nt<1>); break;
    case 2: go(skinny_nt<2>); break;
    case 3: go(skinny_nt<3>); break;
    default: go(skinny_nt<4>); break;
  }
  if (pp) {
    const int n4 = M * N / 4;
    hipLaunchKernelGGL(skinny_reduce, dim3((n4 + 255) / 256), dim3(256), 0, stream, (const float*)pp, nsplit,
                       (unsigned short*)Y, (const unsigned short*)R, ldy, M, N);
  }
  return gs_launch_status();
}
