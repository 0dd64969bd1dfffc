// bf16 GEMM, 4 waves x 128x128 per wave, accumulators pinned in AGPRs (variant 4).
//
// C[M,N] = epilogue(A[M,K] · B[N,K]^T), aligned shapes only (M % 256 == N % 256 == 0,
// K % 128 == 0); the launcher in gemm_bf16.hip checks and falls back otherwise.
//
// Why this shape (profiles/gemm_pmc_8192.md): the 8-wave kernels give every wave a 128x64
// output, so a CU re-reads 48 KiB of LDS per K-tile per SIMD and parks ~29 % of its wave
// cycles at barriers. One wave per SIMD owning 128x128 reads 32 KiB per K-tile (the shape of
// the hipBLASLt kernel) and needs no partner wave, but its 256 fp32 accumulators exceed the
// 256-VGPR architectural file. hipcc, left alone, splits them between VGPRs and AGPRs and
// spills (the former variant 3). Here every MFMA is an inline-asm statement whose C/D operand
// is constrained to the accumulator file ("+a"), so the 64 f32x4 accumulators live in
// a[0:255] for the whole kernel and the fragments, addresses and DMA pointers use ~140 VGPRs.
//
// Pipeline (one raw barrier per 64-deep K-tile, two LDS stages of 64 KiB):
//   phase A(t): 64 MFMA on fragment set 0 (k 0..31 of tile t), interleaved 1 ds_read per 4
//               MFMA filling set 1 (k 32..63 of tile t, buffer t&1)
//   boundary  : s_waitcnt vmcnt(0) lgkmcnt(0)  (tile t+1 landed, set 1 in registers); s_barrier
//   phase B(t): 64 MFMA on set 1, interleaved per 4 MFMA with 1 global_load_lds of tile t+2
//               into buffer t&1 (every wave's reads of it retired before the barrier) and
//               1 ds_read filling set 0 from tile t+1 (buffer (t+1)&1, visible after the barrier)
// Each DMA therefore has two phases (~2k MFMA cycles) to land before its wait.
// The last loop iteration waits for every DMA before the epilogue (s_waitcnt at its boundary).
// LDS image and swizzle as in gemm_bf16.hip (chunk c of row r at c ^ ((r >> 1) & 7)).
//
// Hazards the compiler does not pad around asm (cdna_hip_programming.md §5.7): fragment VGPRs
// are written only by ds_read (hipcc's lgkmcnt covers them — the asm names them as inputs);
// each accumulator is rewritten 64 MFMAs after its previous write; the AGPR zero-init and the
// epilogue's v_accvgpr_read are separated from the MFMA stream by explicit s_nop pads.
#include "common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NT = 256;
constexpr int A_STAGE = BM * BK * 2;   // 32 KiB
constexpr int STAGE = 2 * A_STAGE;     // A + B
constexpr int LDS_BYTES = 2 * STAGE;   // 128 KiB
// Tile rasterisation group height. 4 over 8 for the 4-wave kernel with streamed stores, interleaved
// on one box (profiles/gemm_group_m_ab_w4_r2.jsonl): 4096^3 +1.9 %, 4096x4096x1024 +5.3 %,
// 8192^3 +0.8 %, 16384x4096x4096 +0.5 %, 4096x4096x14336 +0.4 %, 4096x14336x4096 -1.2 %.
constexpr int GROUP_M = 4;

enum { EP_BIAS = 1, EP_SILU = 2, EP_RESID = 4, EP_SWIGLU = 8, EP_STAGED = 16, EP_NT = 32, EP_WT = 64 };   // 16-64: internal only

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

#define MFMA_A(acc, b, a) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a))

struct Frags {
  bf16x8_t a[8], b[8];
};

// 64 MFMAs on fragment set `f` into acc; `extra(g, u)` runs after MFMA u (0..3) of group g
// (0..15), each followed by a scheduling fence so the interleave is exactly the source order.
template <typename Extra>
__device__ __forceinline__ void mfma_phase(f32x4_t (&acc)[8][8], const Frags& f, Extra extra) {
#pragma unroll
  for (int g = 0; g < 16; ++g) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = g * 4 + u, i = idx >> 3, j = idx & 7;
      MFMA_A(acc[i][j], f.b[j], f.a[i]);
      extra(g, u);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Block -> output tile: XCD-aware bijective remap, then GROUP_M rasterisation (as gemm_bf16.hip).
__device__ __forceinline__ void tile_origin(int M, int N, int flags, int& m0, int& n0) {
  const int nbm = M / BM, nbn = N / BN, nwg = nbm * nbn;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int gm = (flags >> 8) & 0xff ? (flags >> 8) & 0xff : GROUP_M;
  const int per_group = gm * nbn;
  const int first_m = (wgid / per_group) * gm;
  const int gsz = min(nbm - first_m, gm);
  m0 = (first_m + (wgid % per_group) % gsz) * BM;
  n0 = ((wgid % per_group) / gsz) * BN;
}

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// One 16-B C store. EP_WT | EP_NT (the default of every epilogue): device scope + streamed, so C is
// written through L2 instead of sitting dirty there until the kernel-end release writes it back
// (4096^3 back to back: 93.8 -> 91.5 us, 8192^3: 698 -> 679 us; profiles/gemm_store_policy_r2.md).
// The s_nop covers the store-data hazard hipcc does not see through asm (a VALU overwriting a
// >8-B store's data VGPRs right after issue).
template <int EPI>
__device__ __forceinline__ void store16(u32x4_t* dst, u32x4_t val) {
  if constexpr ((EPI & EP_WT) != 0 && (EPI & EP_NT) != 0)
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(dst), "v"(val) : "memory");
  else if constexpr ((EPI & EP_WT) != 0)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(val) : "memory");
  else if constexpr ((EPI & EP_NT) != 0)
    __builtin_nontemporal_store(val, dst);
  else
    *dst = val;
}

// Epilogue of a 128x128 wave tile. Lane (row r = lane & 15, quad q = lane >> 4) holds
// C[m][n..n+3] of every 16x16 tile (i, j), m = mbase + 16 i, n = nbase + 16 j + 4 q. After
// + bias, SiLU, + residual (by flags) and bf16 packing, one v_permlane16_swap per dword pairs
// tiles j and j+1: quads 0/2 then hold 8 contiguous columns of tile j (4q .. 4q+7 -> cols 0-7 /
// 8-15), quads 1/3 those of tile j+1, so each lane stores 16 B instead of 2 x 8 B
// (cdna_hip_programming.md T21 with 16-lane rows). Needs ldc % 8 == 0 and a 16-B aligned C.
// EPI (compile-time flags) keeps the epilogue branch-free: with runtime flags hipcc built a
// branchy CFG per element and spilled accumulators into scratch.
template <int EPI>
__device__ __forceinline__ void epilogue_128x128(f32x4_t (&acc)[8][8], unsigned short* __restrict__ C,
                                                 const unsigned short* __restrict__ bias,
                                                 const unsigned short* __restrict__ R, int ldc, int mbase, int nbase,
                                                 int q) {
  const int ncol = nbase - 4 * q + 16 * (q & 1) + 8 * (q >> 1);   // store column of tile pair 0
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mbase + i * 16;
    // the accumulators of row i stay in AGPRs until here: hipcc otherwise copies them all to
    // VGPRs at the loop exit and spills
    asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                 "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      unsigned w[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * jp + h, n = nbase + j * 16;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr ((EPI & EP_BIAS) != 0) {
          const u16x4_t bb = *(const u16x4_t*)(bias + n);
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] += bf16_to_f32(bb[t]);
        }
        if constexpr ((EPI & EP_SILU) != 0) {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = silu_f32(v[t]);
        }
        if constexpr ((EPI & EP_RESID) != 0) {
          const u16x4_t rr = *(const u16x4_t*)(R + (size_t)m * ldc + n);
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] += bf16_to_f32(rr[t]);
        }
        w[h][0] = (unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16);
        w[h][1] = (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const auto r = __builtin_amdgcn_permlane16_swap(w[0][d], w[1][d], false, false);
        w[0][d] = r[0];
        w[1][d] = r[1];
      }
      store16<EPI>((u32x4_t*)(C + (size_t)m * ldc + ncol + 32 * jp), u32x4_t{w[0][0], w[0][1], w[1][0], w[1][1]});
    }
    __builtin_amdgcn_sched_barrier(0);   // one row of tiles at a time: bounds VGPR pressure
  }
}

// Plain epilogue staged through LDS (opt-in, GS_W4_STAGED_EPI=1): each wave writes its 128 x 128
// bf16 tile into its own 32 KiB of the (by then dead) operand buffers, 16-B chunks XOR-swizzled by
// row so the 16 rows a ds_write_b64 touches fall in distinct banks, then streams it out 4 full
// 256-B rows per store instruction (8 whole 128-B lines) instead of 16 rows x 64 B.
__device__ __forceinline__ void epilogue_staged(f32x4_t (&acc)[8][8], unsigned short* __restrict__ C, int ldc,
                                                char* wsmem, int mtile, int ntile, int lane) {
  const int lr = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                 "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
    const int r = lr + 16 * i;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
      const u32x2_t w = {(unsigned)f32_to_bf16(acc[i][j][0]) | ((unsigned)f32_to_bf16(acc[i][j][1]) << 16),
                         (unsigned)f32_to_bf16(acc[i][j][2]) | ((unsigned)f32_to_bf16(acc[i][j][3]) << 16)};
      const int chunk = 2 * j + (q >> 1);
      *(u32x2_t*)(wsmem + r * 256 + ((chunk ^ (r & 15)) << 4) + (q & 1) * 8) = w;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  const int chunk = lane & 15;
#pragma unroll 8
  for (int rb = 0; rb < 32; ++rb) {
    const int r = rb * 4 + (lane >> 4);
    const u32x4_t v = *(const u32x4_t*)(wsmem + r * 256 + ((chunk ^ (r & 15)) << 4));
    *(u32x4_t*)(C + (size_t)(mtile + r) * ldc + ntile + chunk * 8) = v;
  }
}

// SwiGLU epilogue: B's rows are gate/up interleaved in blocks of 16 (rows 32b .. 32b+15 = gate
// features 16b .., rows 32b+16 .. 32b+31 = up features 16b ..), so tiles 2jj / 2jj+1 of a wave
// hold gate / up of the same 16 features and out[m][f] = silu(g) * u is lane-local. The wave
// writes a 128 x 64 feature tile of the [M, N/2] output (ldc in features); pairs of feature
// tiles are merged by v_permlane16_swap into 16-B stores as in epilogue_128x128. Saves writing
// and re-reading the [M, N] gate|up activations (the separate silu_mul pass).
template <int EPI>
__device__ __forceinline__ void epilogue_swiglu(f32x4_t (&acc)[8][8], unsigned short* __restrict__ C, int ldc,
                                                int mbase, int fbase, int q) {
  const int fcol = fbase + 16 * (q & 1) + 8 * (q >> 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mbase + i * 16;
    asm volatile("" : "+a"(acc[i][0]), "+a"(acc[i][1]), "+a"(acc[i][2]), "+a"(acc[i][3]), "+a"(acc[i][4]),
                 "+a"(acc[i][5]), "+a"(acc[i][6]), "+a"(acc[i][7]));
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      unsigned w[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int jj = 2 * jp + h;
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = silu_f32(acc[i][2 * jj][t]) * acc[i][2 * jj + 1][t];
        w[h][0] = (unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16);
        w[h][1] = (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const auto r = __builtin_amdgcn_permlane16_swap(w[0][d], w[1][d], false, false);
        w[0][d] = r[0];
        w[1][d] = r[1];
      }
      store16<EPI>((u32x4_t*)(C + (size_t)m * ldc + fcol + 32 * jp), u32x4_t{w[0][0], w[0][1], w[1][0], w[1][1]});
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// DMA_GROUPS: the 16 DMA instructions of a phase B go 16 / DMA_GROUPS at a time into MFMA groups
// DMA_G0 .. DMA_G0 + DMA_GROUPS - 1 (earlier issue = more time to land before the next boundary's
// wait). The 16 fragment reads of each phase go two per group into 8 consecutive groups (phase A:
// 0-7; phase B: RDB_G0 .. RDB_G0 + 7, so DMA and reads can be kept apart in LDS time), after MFMAs
// RD_U0 and RD_U1 of the group; a DMA follows MFMA DMA_U.
// NSTG (0, 4 or 8): the last NSTG of the 16 pieces of a K-tile (B rows) skip the LDS DMA: they are
// loaded into VGPRs during phase A (buffer_load_dwordx4, one per group from group 0) and written
// to the same LDS image in phase B (ds_write_b128, lane-linear like the DMA, conflict-free), in
// the groups between the remaining DMA pieces. The boundary wait then leaves those NSTG loads in
// flight (vmcnt(NSTG)).
// KV (schedule 12 only): the K-tile offset goes into the per-lane VGPR offset (one v_add per operand
// and tile) and the scalar offset is the loop-invariant row offset i * 32 rows, instead of an s_add
// per DMA piece: 14 fewer SALU per K-tile, yet measured 0.6 % faster at 4096^3 and 1-2 % slower at
// 8192^3, long K and N = 14336 (order-rotated sweep, profiles/gemm_kv_offset_r2_rotated.json).
template <int DMA_GROUPS, int RD_U0, int RD_U1, int DMA_U, int EPI, int DMA_G0 = 0, int RDB_G0 = 0, int NSTG = 0,
          int KV = 0>
__global__ __launch_bounds__(NT, 1) void gemm_bf16_nt_w4a(
    const unsigned short* __restrict__ A, const unsigned short* __restrict__ B, unsigned short* __restrict__ C,
    const unsigned short* __restrict__ bias, const unsigned short* __restrict__ R, int M, int N, int K, int lda,
    int ldb, int ldc, int flags) {
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int m0, n0;
  tile_origin(M, N, flags, m0, n0);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably uniform -> SGPR
  const int wm = wave >> 1, wn = wave & 1;

  // ---- DMA: instruction i (0..7) of wave w fills rows (i*4 + w)*8 + lane/8 of an operand
  // image (1 KiB per instruction); lane's chunk slot lane%8 <- logical chunk swz(row, lane%8),
  // which is the same for every i because i*32 rows shift (row >> 1) & 7 by a multiple of 8.
  const int drow = wave * 8 + (lane >> 3);
  const int dc = swz(drow, lane & 7);
  // Buffer descriptors over this block's 256 rows of A and B (base and size from kernel
  // arguments and blockIdx only, so they stay in SGPRs); the per-lane part is one VGPR offset,
  // the DMA index i and the K-tile go into the scalar soffset, so a DMA costs no VALU.
  // In the last two K-tiles the DMA slot has no tile left to fetch: it runs on zero-size descriptors
  // (every lane out of range, so no memory traffic and nothing for the final vmcnt wait to cover).
  const __amdgpu_buffer_rsrc_t rA_live =
      __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * lda), (short)0, BM * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB_live =
      __builtin_amdgcn_make_buffer_rsrc((void*)(B + (size_t)n0 * ldb), (short)0, BN * ldb * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rA_dead = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB_dead = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0, 0x00020000);
  __amdgpu_buffer_rsrc_t rA = rA_live, rB = rB_live;
  const unsigned voffA = (unsigned)(drow * lda + dc * 8) * 2u;
  const unsigned voffB = (unsigned)(drow * ldb + dc * 8) * 2u;
  const unsigned a32 = 64u * lda, b32 = 64u * ldb;   // bytes of 32 rows
  char* const wdst = smem + wave * 1024;   // + buf*STAGE + i*4096 (+ A_STAGE for B)

  // DMA instruction g (0..15) of K-tile kt into buffer buf: g < 8 -> A rows, else B rows
  auto dma = [&](int buf, int kt, int g) {
    const int i = g & 7;
    const unsigned koff = (unsigned)kt * (BK * 2);
    const unsigned va = KV ? voffA + koff : voffA, vb = KV ? voffB + koff : voffB;
    const unsigned sa = KV ? i * a32 : i * a32 + koff, sb = KV ? i * b32 : i * b32 + koff;
    if (g < 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rA, (__attribute__((address_space(3))) void*)(wdst + buf * STAGE + i * 4096), 16, va, sa, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rB, (__attribute__((address_space(3))) void*)(wdst + buf * STAGE + A_STAGE + i * 4096), 16, vb, sb, 0, 0);
  };

  static_assert(NSTG == 0 || NSTG == 4 || NSTG == 8, "NSTG: 0, 4 or 8 staged B pieces");
  u32x4_t stg[NSTG > 0 ? NSTG : 1];
  // staged piece s = DMA piece 16 - NSTG + s (B rows i = that & 7), same global bytes and LDS slot
  auto stage_load = [&](int kt, int s) {
    const int i = (16 - NSTG + s) & 7;
    stg[s] = __builtin_amdgcn_raw_buffer_load_b128(rB, (int)voffB, (int)(i * b32 + (unsigned)kt * (BK * 2)), 0);
  };
  auto stage_write = [&](int buf, int s) {
    const int i = (16 - NSTG + s) & 7;
    *(u32x4_t*)(wdst + buf * STAGE + A_STAGE + i * 4096 + lane * 16) = stg[s];
  };

  // ---- fragment addressing: lane reads row (lane & 15) of a 16-row tile, k-chunk
  // kk*4 + lane/16; the swizzle term depends only on lane & 15 (tile bases are multiples of 16)
  const int lr = lane & 15;
  const int co0 = swz(lr, lane >> 4) << 4;
  const int co1 = swz(lr, 4 + (lane >> 4)) << 4;
  const int a_off = (wm * 128 + lr) * 128;
  const int b_off = A_STAGE + (wn * 128 + lr) * 128;
  // read g (0..15) of a fragment set from buffer buf: g < 8 -> B tile g, else A tile g-8
  auto frag_read = [&](Frags& f, int buf, int co, int g) {
    const char* base = smem + buf * STAGE + co;
    if (g < 8)
      f.b[g] = *(const bf16x8_t*)(base + b_off + g * 2048);
    else
      f.a[g - 8] = *(const bf16x8_t*)(base + a_off + (g - 8) * 2048);
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  Frags f0, f1;
  const int KT = K / BK;   // even, >= 2

  // ---- prologue: tiles 0 and 1 in flight, wait for tile 0, read set 0 of tile 0 ----
#pragma unroll
  for (int g = 0; g < 16; ++g) dma(0, 0, g);
#pragma unroll
  for (int g = 0; g < 16; ++g) dma(1, 1, g);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int g = 0; g < 16; ++g) frag_read(f0, 0, co0, g);
  __builtin_amdgcn_sched_barrier(0);

  // One loop body for every tile, so the accumulators keep one register assignment (a peeled
  // tail made hipcc shuffle them through VGPRs). Past the end, the DMA runs on the zero-size
  // descriptors (zeros into the buffer just released) and phase B reads a dead fragment set.
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    const int kdma = min(kt + 2, KT - 1);
    if (kt + 2 >= KT) {
      rA = rA_dead;
      rB = rB_dead;
    }
    // hipcc may place the accumulators' zero-init (v_accvgpr_write) right before the loop:
    // 2 wait states before an MFMA reads them as srcC (2 cycles per 4k-cycle iteration)
    asm volatile("s_nop 1" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // phase A: set-1 reads; the boundary wait sits between the last two MFMAs and the barrier
    // after the last one, so the matrix pipe stays busy while the wave waits
    mfma_phase(acc, f0, [&](int g, int u) {
      if (NSTG > 0 && g < NSTG && u == 0) stage_load(kdma, g);
      if (g < 8 && u == RD_U0) frag_read(f1, buf, co1, 2 * g);
      if (g < 8 && u == RD_U1) frag_read(f1, buf, co1, 2 * g + 1);
      if (g == 15 && u == 2) {
        if constexpr (NSTG == 8)
          asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else if constexpr (NSTG == 4)
          asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      if (g == 15 && u == 3) __builtin_amdgcn_s_barrier();
    });
    // phase B: DMA of tile kt+2 into the buffer just released, set-0 reads of tile kt+1
    mfma_phase(acc, f1, [&](int g, int u) {
      if constexpr (NSTG > 0) {
        constexpr int step = 16 / NSTG;   // every step-th group writes a staged piece
        if (u == DMA_U && g % step == step - 1) stage_write(buf, g / step);
        else if (u == DMA_U) dma(buf, kdma, g - g / step);
      } else if (u == DMA_U && g >= DMA_G0 && g < DMA_G0 + DMA_GROUPS) {
#pragma unroll
        for (int d = 0; d < 16 / DMA_GROUPS; ++d) dma(buf, kdma, (g - DMA_G0) * (16 / DMA_GROUPS) + d);
      }
      if (g >= RDB_G0 && g < RDB_G0 + 8 && u == RD_U0) frag_read(f0, buf ^ 1, co0, 2 * (g - RDB_G0));
      if (g >= RDB_G0 && g < RDB_G0 + 8 && u == RD_U1) frag_read(f0, buf ^ 1, co0, 2 * (g - RDB_G0) + 1);
    });
    // last MFMA D -> whatever reads the accumulators next: hipcc places its AGPR copies for
    // the epilogue on the loop-exit edge, ahead of any statement after the loop, so the pad
    // must be inside the final iteration
    if (kt == KT - 1) asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  }

  if constexpr ((EPI & EP_STAGED) != 0) {
    // the operand buffers are dead once every wave is past its last fragment read and the
    // (zero-size) tail DMAs have landed
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    epilogue_staged(acc, C, ldc, smem + wave * 32768, m0 + wm * 128, n0 + wn * 128, lane);
  } else if constexpr ((EPI & EP_SWIGLU) != 0)
    epilogue_swiglu<EPI>(acc, C, ldc, m0 + wm * 128 + lr, (n0 + wn * 128) / 2, lane >> 4);
  else
    epilogue_128x128<EPI>(acc, C, bias, R, ldc, m0 + wm * 128 + lr, n0 + wn * 128 + (lane >> 4) * 4, lane >> 4);
}

constexpr int W4_SCHEDS = 16;
int g_w4_sched = 0;

}  // namespace

// Phase-B schedule of the plain 4-wave product (0 = default; 1..15 = the alternatives listed in
// gs_gemm_w4_launch) for A/B sweeps (tools/gemm_sched_sweep.py).
GS_KERNEL_API int gs_gemm_w4_set_sched(int s) {
  if (s < 0 || s >= W4_SCHEDS) return GS_EINVAL;
  g_w4_sched = s;
  return GS_OK;
}

// Launch the 4-wave kernel; the caller (gs_gemm_bf16_nt) has validated pointers/strides/flags.
// Returns GS_EINVAL when the shape or output layout does not suit it (the caller falls back).
int gs_gemm_w4_launch(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                      int lda, int ldb, int ldc, int flags, hipStream_t stream, int reps) {
  if (reps < 1 || reps > 65535) return GS_EINVAL;
  if (M % BM || N % BN || K % (2 * BK)) return GS_EINVAL;
  if ((size_t)BM * lda * 2 > 0xffffffffu || (size_t)BN * ldb * 2 > 0xffffffffu) return GS_EINVAL;
  if (ldc % 8 || ((uintptr_t)C & 15)) return GS_EINVAL;   // 16-B epilogue stores
  // DMA after MFMA 1 of each group, the two fragment reads after MFMAs 2 and 3 of groups 0-7:
  // the best of the placements swept on MI355X (profiles/gemm_w4_variants.md)
  using Kern = void (*)(const unsigned short*, const unsigned short*, unsigned short*, const unsigned short*,
                       const unsigned short*, int, int, int, int, int, int, int);
  constexpr int ST = EP_WT | EP_NT;   // C store policy of every default kernel (store16)
  static const Kern kerns[10] = {gemm_bf16_nt_w4a<16, 2, 3, 1, ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, 1 | ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, 2 | ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, 3 | ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, 4 | ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, 5 | ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, 6 | ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, 7 | ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, EP_SWIGLU | ST, 0, 0, 0, 0>,
                                gemm_bf16_nt_w4a<16, 2, 3, 1, EP_STAGED, 0, 0, 0, 0>};
  // Alternative placements of phase B's DMA and fragment reads for the plain product (schedule
  // sweeps, gs_gemm_w4_set_sched): <DMA groups, first DMA group, first read group of phase B>
  static const Kern sched[W4_SCHEDS] = {
      gemm_bf16_nt_w4a<16, 2, 3, 1, ST, 0, 0, 0, 0>,   // 0: default (DMA spread over 16 groups, reads 0-7, ST stores)
      gemm_bf16_nt_w4a<8, 2, 3, 1, 0, 0, 8>,    // 1: DMA in groups 0-7, reads 8-15
      gemm_bf16_nt_w4a<16, 2, 3, 1, 0, 0, 4>,   // 2: DMA spread, reads 4-11
      gemm_bf16_nt_w4a<8, 2, 3, 1, 0, 0, 4>,    // 3: DMA in groups 0-7, reads 4-11
      gemm_bf16_nt_w4a<8, 2, 3, 1, 0, 8, 0>,    // 4: reads 0-7, DMA in groups 8-15
      gemm_bf16_nt_w4a<16, 2, 3, 1, 0, 0, 8>,   // 5: DMA spread, reads 8-15
      gemm_bf16_nt_w4a<16, 2, 3, 1, EP_NT, 0, 0>,   // 6: 0 with non-temporal C stores
      gemm_bf16_nt_w4a<16, 2, 3, 1, EP_NT, 0, 8>,   // 7: 5 with non-temporal C stores
      gemm_bf16_nt_w4a<16, 2, 3, 1, EP_WT, 0, 0>,   // 8: 0 with device-scope (write-through) C stores
      gemm_bf16_nt_w4a<16, 2, 3, 1, 0, 0, 0>,   // 9: plain (write-back) C stores, scalar K offsets
      gemm_bf16_nt_w4a<16, 2, 3, 1, ST, 0, 0, 8>,   // 10: 0 with B staged through VGPRs (A by DMA)
      gemm_bf16_nt_w4a<16, 2, 3, 1, ST, 0, 0, 4>,   // 11: 0 with half of B staged through VGPRs
      gemm_bf16_nt_w4a<16, 2, 3, 1, ST, 0, 0, 0, 1>,   // 12: 0 with the K offset in the VGPR offset (KV)
      gemm_bf16_nt_w4a<16, 2, 3, 0, ST>,   // 13: 0 with the DMA after MFMA 0 of its group
      gemm_bf16_nt_w4a<16, 1, 2, 3, ST>,   // 14: reads after MFMAs 1 / 2, DMA after MFMA 3
      gemm_bf16_nt_w4a<16, 0, 1, 2, ST>,   // 15: reads after MFMAs 0 / 1, DMA after MFMA 2
  };
  static const bool staged = [] {
    const char* e = getenv("GS_W4_STAGED_EPI");
    return e != nullptr && e[0] == '1';
  }();
  if ((flags & EP_SWIGLU) && (flags & 7)) return GS_EINVAL;   // SwiGLU takes no other epilogue
  Kern kern = kerns[(flags & EP_SWIGLU) ? 8 : (flags & 7) ? (flags & 7) : staged ? 9 : 0];
  if (kern == kerns[0] && g_w4_sched > 0) kern = sched[g_w4_sched];
  static bool attr_set = false;
  if (!attr_set) {
    for (Kern k : kerns)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    for (Kern k : sched)
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr_set = true;
  }
  const int nblocks = (M / BM) * (N / BN);
  // reps > 1: the same GEMM `reps` times in one dispatch (grid.y; tile_origin reads blockIdx.x only),
  // so back-to-back repetitions refill CUs as workgroups retire instead of draining at each kernel
  // boundary. Every repetition computes the full product and stores identical values to C.
  kern<<<dim3(nblocks, reps), dim3(NT), LDS_BYTES, stream>>>(
      (const unsigned short*)A, (const unsigned short*)B, (unsigned short*)C, (const unsigned short*)bias,
      (const unsigned short*)R, M, N, K, lda, ldb, ldc, flags);
  return gs_launch_status();
}
