// bf16 GEMM on CDNA4 matrix cores: C[M,N] = epilogue(A[M,K] · B[N,K]^T)
//
// "NT" layout = torch.nn.functional.linear (activations [M,K], weights [N,K], both
// K-contiguous), the shape of every projection in the demo workloads and of the bin-pack
// traffic generator.
//
// Design (cdna_hip_programming.md §5, measured guidance for gfx950):
//  * 256x256 block tile, BK = 64, 8 waves (2 along M x 4 along N), each wave 128x64 =
//    8x4 tiles of v_mfma_f32_16x16x32_bf16 (fp32 accumulators, 128 regs/lane);
//  * operands staged global -> LDS with global_load_lds_dwordx4 (no VGPR round trip), two
//    64 KiB stages (128 KiB LDS, one block per CU, all LDS in ONE __shared__ array so hipcc
//    does not drain the DMA before every ds_read);
//  * the LDS image is lane-linear (a DMA writes base + lane*16), so the bank-conflict
//    swizzle is applied on the SOURCE address and undone on the ds_read address: chunk c of
//    row r lives at chunk c ^ ((r >> 1) & 7) of its 128-B row, which makes every 16-lane
//    ds_read_b128 group hit 16 distinct 16-B slots of the 256-B bank row;
//  * MFMA operands are swapped (weights as the "A" operand) so each lane's 4 accumulator
//    registers are 4 consecutive output columns: 8-byte packed bf16 stores;
//  * XCD-aware bijective block remap + GROUP_M rasterisation so the 8 blocks that share an
//    XCD's L2 share A panels;
//  * fused epilogue: + bias[n], SiLU, + residual[m,n] (flags), bf16 output; SwiGLU (flag 8,
//    gate/up rows interleaved by 16) only on the 4-wave kernel of gemm_bf16_w4.hip.
// Requirements (checked by the launcher): K % 64 == 0, lda/ldb % 8 == 0, 16-B aligned A/B,
// N % 4 == 0, ldc % 4 == 0.
// Aligned shapes (M, N % 256, K % 128) run the 4-wave kernel of gemm_bf16_w4.hip (AGPR
// accumulators, 128x128 per wave); the two 8-wave kernels here cover the rest.
#include "common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NTHREADS = 512;
constexpr int A_STAGE = BM * BK * 2;          // 32 KiB
constexpr int B_STAGE = BN * BK * 2;          // 32 KiB
constexpr int STAGE = A_STAGE + B_STAGE;      // 64 KiB
constexpr int LDS_BYTES = 2 * STAGE;          // 128 KiB
constexpr int GROUP_M = 8;

enum { EP_BIAS = 1, EP_SILU = 2, EP_RESID = 4, EP_SWIGLU = 8 };

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__global__ __launch_bounds__(NTHREADS, 2) void gemm_bf16_nt_256(
    const unsigned short* __restrict__ A, const unsigned short* __restrict__ B, unsigned short* __restrict__ C,
    const unsigned short* __restrict__ bias, const unsigned short* __restrict__ R, int M, int N, int K, int lda,
    int ldb, int ldc, int flags) {
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // ---- tile assignment: XCD-aware bijective remap, then GROUP_M rasterisation ----
  const int nbm = (M + BM - 1) / BM, nbn = (N + BN - 1) / BN, nwg = nbm * nbn;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int gm = (flags >> 8) & 0xff ? (flags >> 8) & 0xff : GROUP_M;   // rasterisation group (rows)
  const int per_group = gm * nbn;
  const int first_m = (wgid / per_group) * gm;
  const int gsz = min(nbm - first_m, gm);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;

  // ---- DMA source pointers: 4 instructions for A, 4 for B per stage ----
  // instruction i of wave w writes LDS bytes [(i*8 + w) * 1024, +1024) = 8 rows x 128 B;
  // lane l lands at row (i*8+w)*8 + l/8, chunk slot l%8 which holds logical chunk swz(row, l%8).
  const unsigned short* srcA[4];
  const unsigned short* srcB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (i * 8 + wave) * 8 + (lane >> 3);
    const int c = swz(row, lane & 7);
    const int ga = min(m0 + row, M - 1), gb = min(n0 + row, N - 1);
    srcA[i] = A + (size_t)ga * lda + c * 8;
    srcB[i] = B + (size_t)gb * ldb + c * 8;
  }
  char* const ldsA0 = smem;
  char* const ldsB0 = smem + A_STAGE;

  auto stage = [&](int buf, int kt) {
    char* a = ldsA0 + buf * STAGE;
    char* b = ldsB0 + buf * STAGE;
    const int koff = kt * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(srcA[i] + koff, a + (i * 8 + wave) * 1024);
      glds16(srcB[i] + koff, b + (i * 8 + wave) * 1024);
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment row offsets (bytes) inside a stage
  const int arow0 = wm * 128 + (lane & 15);
  const int brow0 = wn * 64 + (lane & 15);
  const int csub = lane >> 4;  // which 8-element k chunk inside a 32-wide MFMA k-step

  const int KT = K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) stage(cur ^ 1, kt + 1);
    const char* a = ldsA0 + cur * STAGE;
    const char* b = ldsB0 + cur * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + csub;
      bf16x8_t af[8], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = brow0 + j * 16;
        bfr[j] = *(const bf16x8_t*)(b + row * 128 + (swz(row, c) << 4));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = arow0 + i * 16;
        af[i] = *(const bf16x8_t*)(a + row * 128 + (swz(row, c) << 4));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          // weights as the first operand: D[n][m] -> lane holds 4 consecutive n of one m
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue: lane holds C[m][n..n+3], m = .. + (lane&15), n = .. + (lane>>4)*4 ----
  const int mbase = m0 + wm * 128 + (lane & 15);
  const int nbase = n0 + wn * 64 + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mbase + i * 16;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nbase + j * 16;
      if (n >= N) continue;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (flags & EP_BIAS) {
        const u16x4_t bb = *(const u16x4_t*)(bias + n);
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] += bf16_to_f32(bb[t]);
      }
      if (flags & EP_SILU) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = silu_f32(v[t]);
      }
      if (flags & EP_RESID) {
        const u16x4_t rr = *(const u16x4_t*)(R + (size_t)m * ldc + n);
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] += bf16_to_f32(rr[t]);
      }
      u16x4_t o;
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = f32_to_bf16(v[t]);
      *(u16x4_t*)(C + (size_t)m * ldc + n) = o;
    }
  }
}


// ---------------------------------------------------------------------------------------
// v2: ping-pong 8-phase schedule (aligned shapes: M % 256 == 0, N % 256 == 0, K % 128 == 0)
//
// Same 256x256 tile / 8 waves / 16x16x32 MFMA as above; what changes is the pipeline.
//  * LDS = 2 buffers (even / odd K-tile) x 4 quarter slots of 16 KiB. A quarter holds one
//    operand's rows for one half of every wave's sub-tile: A-mh (rows wm*128 + mh*64 + 0..63
//    for wm = 0, 1) and B-nh (n-rows wn*64 + nh*32 + 0..31 for wn = 0..3). Per K-tile a wave
//    walks its 128x64 output in 4 quadrant phases (mh, nh) = (0,0), (0,1), (1,1), (1,0),
//    reading A0+B0, B1, A1, B0 — so every quarter is last read in exactly ONE phase and can be
//    restaged by the very next phase (its reads were retired by lgkmcnt(0) before that phase's
//    first barrier).
//  * one quarter (2 x global_load_lds_dwordx4 per thread) is staged per phase; the K-loop runs
//    two K-tiles (8 phases) per iteration and waits s_waitcnt vmcnt(6) only in phases 4 and 8,
//    keeping 3 quarters (~1500 MFMA cycles) of prefetch in flight across raw s_barriers, and a
//    buffer is first read one barrier after the wait that retires it
//    (cdna_hip_programming.md "Pipelining across barriers").
//  * the two wave groups (wm = 0 / 1 — one of each on every SIMD, waves go to SIMDs
//    cyclically) run one barrier apart: while one wave issues its ds_reads + DMA, the other
//    wave on the SIMD issues its 16 MFMAs, so the matrix pipe alternates between them.
// Staging order per iteration i (tiles 2i, 2i+1; buffer b = tile & 1):
//   P1 (2i+1,B0)  P2 (2i+2,A0)  P3 (2i+2,B1)  P4 (2i+2,A1) + vmcnt(6) -> tile 2i+1 landed
//   P5 (2i+2,B0)  P6 (2i+3,A0)  P7 (2i+3,B1)  P8 (2i+3,A1) + vmcnt(6) -> tile 2i+2 landed
constexpr int QBYTES = 128 * BK * 2;   // 16 KiB quarter
enum { QA0 = 0, QA1 = 1, QB0 = 2, QB1 = 3 };

__device__ __forceinline__ void sched_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void raw_barrier() {
  sched_fence();
  __builtin_amdgcn_s_barrier();
  sched_fence();
}

struct PPState {
  const unsigned short* srcA[2];   // per DMA instruction, quarter h = 0 (h = 1: + 64 rows)
  const unsigned short* srcB[2];   // per DMA instruction, quarter h = 0 (h = 1: + 32 rows)
  size_t a_h1, b_h1;               // element offsets of the h = 1 quarter
  char* lds;
  int wave;
};

// DMA one quarter (q) of K-tile kt into buffer (kt & 1).
__device__ __forceinline__ void pp_stage(const PPState& st, int q, int kt) {
  char* slot = st.lds + ((kt & 1) * 4 + q) * QBYTES;
  const int koff = kt * BK;
  const bool isA = q < 2;
  const size_t hoff = (q & 1) ? (isA ? st.a_h1 : st.b_h1) : 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const unsigned short* src = (isA ? st.srcA[i] : st.srcB[i]) + hoff + koff;
    glds16(src, slot + (i * 8 + st.wave) * 1024);
  }
}

__global__ __launch_bounds__(NTHREADS, 2) void gemm_bf16_nt_256_pp(
    const unsigned short* __restrict__ A, const unsigned short* __restrict__ B, unsigned short* __restrict__ C,
    const unsigned short* __restrict__ bias, const unsigned short* __restrict__ R, int M, int N, int K, int lda,
    int ldb, int ldc, int flags) {
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nbm = M / BM, nbn = N / BN, nwg = nbm * nbn;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int gm = (flags >> 8) & 0xff ? (flags >> 8) & 0xff : GROUP_M;   // rasterisation group (rows)
  const int per_group = gm * nbn;
  const int first_m = (wgid / per_group) * gm;
  const int gsz = min(nbm - first_m, gm);
  const int tm = first_m + (wgid % per_group) % gsz;
  const int tn = (wgid % per_group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;

  PPState st;
  st.lds = smem;
  st.wave = wave;
  st.a_h1 = (size_t)64 * lda;
  st.b_h1 = (size_t)32 * ldb;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    // DMA instruction i of wave w fills quarter-local rows (i*8 + w)*8 + lane/8, chunk slot lane%8
    const int rho = (i * 8 + wave) * 8 + (lane >> 3);
    const int c = swz(rho, lane & 7);
    const int arow = m0 + (rho >> 6) * 128 + (rho & 63);
    const int brow = n0 + (rho >> 5) * 64 + (rho & 31);
    st.srcA[i] = A + (size_t)arow * lda + c * 8;
    st.srcB[i] = B + (size_t)brow * ldb + c * 8;
  }

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // fragment addressing inside a quarter: row rho = base + tile*16 + (lane & 15); the swizzle
  // term ((rho >> 1) & 7) depends only on lane & 15 because base and tile*16 are multiples of 16
  const int lr = lane & 15;
  const int co0 = (swz(lr, 0 * 4 + (lane >> 4))) << 4;
  const int co1 = (swz(lr, 1 * 4 + (lane >> 4))) << 4;
  const int a_lane = (wm * 64 + lr) * 128;
  const int b_lane = (wn * 32 + lr) * 128;

  bf16x8_t af[4][2], bfr[2][2];

  auto readA = [&](int buf, int h) {
    const char* qb = smem + (buf * 4 + (h ? QA1 : QA0)) * QBYTES + a_lane;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *(const bf16x8_t*)(qb + i * 16 * 128 + co0);
      af[i][1] = *(const bf16x8_t*)(qb + i * 16 * 128 + co1);
    }
  };
  auto readB = [&](int buf, int h) {
    const char* qb = smem + (buf * 4 + (h ? QB1 : QB0)) * QBYTES + b_lane;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bfr[j][0] = *(const bf16x8_t*)(qb + j * 16 * 128 + co0);
      bfr[j][1] = *(const bf16x8_t*)(qb + j * 16 * 128 + co1);
    }
  };
  auto mfma_q = [&](int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh * 4 + i][nh * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // one phase: [reads + DMA (+ counted wait)] lgkmcnt(0) barrier [16 MFMA] barrier
#define PP_PHASE(READS, STAGE, WAIT, MH, NH)          \
  do {                                                \
    READS;                                            \
    STAGE;                                            \
    WAIT;                                             \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    raw_barrier();                                    \
    mfma_q(MH, NH);                                   \
    raw_barrier();                                    \
  } while (0)

  const int KT = K / BK;   // even, >= 2
  // prologue: tile 0 (all quarters) into buffer 0, tile 1 minus B0 into buffer 1
  pp_stage(st, QA0, 0);
  pp_stage(st, QB1, 0);
  pp_stage(st, QA1, 0);
  pp_stage(st, QB0, 0);
  pp_stage(st, QA0, 1);
  pp_stage(st, QB1, 1);
  pp_stage(st, QA1, 1);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  raw_barrier();
  if (wm == 1) raw_barrier();   // stagger: wave group 1 runs one barrier behind group 0

  const int iters = KT / 2;
  for (int it = 0; it < iters - 1; ++it) {
    const int t0 = 2 * it;
    PP_PHASE((readA(0, 0), readB(0, 0)), pp_stage(st, QB0, t0 + 1), (void)0, 0, 0);
    PP_PHASE(readB(0, 1), pp_stage(st, QA0, t0 + 2), (void)0, 0, 1);
    PP_PHASE(readA(0, 1), pp_stage(st, QB1, t0 + 2), (void)0, 1, 1);
    PP_PHASE(readB(0, 0), pp_stage(st, QA1, t0 + 2), asm volatile("s_waitcnt vmcnt(6)" ::: "memory"), 1, 0);
    PP_PHASE((readA(1, 0), readB(1, 0)), pp_stage(st, QB0, t0 + 2), (void)0, 0, 0);
    PP_PHASE(readB(1, 1), pp_stage(st, QA0, t0 + 3), (void)0, 0, 1);
    PP_PHASE(readA(1, 1), pp_stage(st, QB1, t0 + 3), (void)0, 1, 1);
    PP_PHASE(readB(1, 0), pp_stage(st, QA1, t0 + 3), asm volatile("s_waitcnt vmcnt(6)" ::: "memory"), 1, 0);
  }
  {  // last iteration: only tile KT-1's B0 is still to be staged
    const int t0 = 2 * (iters - 1);
    PP_PHASE((readA(0, 0), readB(0, 0)), pp_stage(st, QB0, t0 + 1), (void)0, 0, 0);
    PP_PHASE(readB(0, 1), (void)0, (void)0, 0, 1);
    PP_PHASE(readA(0, 1), (void)0, (void)0, 1, 1);
    PP_PHASE(readB(0, 0), (void)0, asm volatile("s_waitcnt vmcnt(0)" ::: "memory"), 1, 0);
    PP_PHASE((readA(1, 0), readB(1, 0)), (void)0, (void)0, 0, 0);
    PP_PHASE(readB(1, 1), (void)0, (void)0, 0, 1);
    PP_PHASE(readA(1, 1), (void)0, (void)0, 1, 1);
    PP_PHASE(readB(1, 0), (void)0, (void)0, 1, 0);
  }
#undef PP_PHASE
  if (wm == 0) raw_barrier();   // balance the stagger barrier

  const int mbase = m0 + wm * 128 + lr;
  const int nbase = n0 + wn * 64 + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mbase + i * 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nbase + j * 16;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (flags & EP_BIAS) {
        const u16x4_t bb = *(const u16x4_t*)(bias + n);
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] += bf16_to_f32(bb[t]);
      }
      if (flags & EP_SILU) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = silu_f32(v[t]);
      }
      if (flags & EP_RESID) {
        const u16x4_t rr = *(const u16x4_t*)(R + (size_t)m * ldc + n);
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] += bf16_to_f32(rr[t]);
      }
      u16x4_t o;
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = f32_to_bf16(v[t]);
      *(u16x4_t*)(C + (size_t)m * ldc + n) = o;
    }
  }
}

int g_group_m = 0;   // 0 = GROUP_M; else tile-rasterisation group height (passed in flags bits 8..15)
int g_variant = 0;   // 0 = auto, 1 = v1 (2-stage, 8 waves), 2 = v2 (ping-pong), 4 = 4-wave AGPR kernel

}  // namespace

// The GEMM-player path: C = A * B^T repeated `reps` times in one dispatch of the 4-wave kernel
// (aligned shapes, no epilogue). GS_EINVAL when the shape does not suit it (caller loops instead).
GS_KERNEL_API int gs_gemm_bf16_nt_repeat(const void* A, const void* B, void* C, int M, int N, int K, int lda,
                                         int ldb, int ldc, int reps, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || lda % 8 || ldb % 8 || lda < K || ldb < K || ldc < N ||
      ((uintptr_t)A & 15) || ((uintptr_t)B & 15))
    return GS_EINVAL;
  return gs_gemm_w4_launch(A, B, C, nullptr, nullptr, M, N, K, lda, ldb, ldc, g_group_m << 8, stream, reps);
}

GS_KERNEL_API int gs_gemm_bf16_nt(const void* A, const void* B, void* C, const void* bias, const void* R, int M,
                                  int N, int K, int lda, int ldb, int ldc, int flags, hipStream_t stream) {
  const bool swiglu = flags & EP_SWIGLU;   // out[M, N/2] = silu(gate) * up, gate/up rows interleaved by 16
  if (M <= 0 || N <= 0 || K <= 0 || K % BK || lda % 8 || ldb % 8 || ldc % 4 || N % 4 || lda < K || ldb < K ||
      ldc < (swiglu ? N / 2 : N) || ((uintptr_t)A & 15) || ((uintptr_t)B & 15) || ((uintptr_t)C & 7))
    return GS_EINVAL;
  if ((flags & EP_BIAS) && !bias) return GS_EINVAL;
  flags = (flags & 0xff) | (g_group_m << 8);
  if (swiglu)   // only the 4-wave kernel has the SwiGLU epilogue (aligned shapes)
    return g_variant == 0 || g_variant == 4 ? gs_gemm_w4_launch(A, B, C, bias, R, M, N, K, lda, ldb, ldc, flags, stream)
                                            : GS_EINVAL;
  if ((flags & EP_RESID) && !R) return GS_EINVAL;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_256, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_256_pp, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    attr_set = true;
  }
  const bool aligned = M % BM == 0 && N % BN == 0 && K % (2 * BK) == 0;
  if (aligned && (g_variant == 0 || g_variant == 4)) {   // 4-wave kernel first when it applies
    const int rc = gs_gemm_w4_launch(A, B, C, bias, R, M, N, K, lda, ldb, ldc, flags, stream);
    if (rc != GS_EINVAL) return rc;
  }
  const int nblocks = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (aligned && g_variant != 1) {
    gemm_bf16_nt_256_pp<<<dim3(nblocks), dim3(NTHREADS), LDS_BYTES, stream>>>(
        (const unsigned short*)A, (const unsigned short*)B, (unsigned short*)C, (const unsigned short*)bias,
        (const unsigned short*)R, M, N, K, lda, ldb, ldc, flags);
    return gs_launch_status();
  }
  hipLaunchKernelGGL(gemm_bf16_nt_256, dim3(nblocks), dim3(NTHREADS), LDS_BYTES, stream,
                     (const unsigned short*)A, (const unsigned short*)B, (unsigned short*)C,
                     (const unsigned short*)bias, (const unsigned short*)R, M, N, K, lda, ldb, ldc, flags);
  return gs_launch_status();
}

// Kernel selection for A/B measurement and tests: 0 = auto (4-wave kernel when it applies, else
// ping-pong when aligned, else 2-stage), 1 = 2-stage only, 2 = ping-pong when aligned, 4 = 4-wave
// when it applies (gemm_bf16_w4.hip), else as 2.
GS_KERNEL_API int gs_gemm_set_variant(int v) {
  if (v < 0 || v > 4 || v == 3) return GS_EINVAL;
  g_variant = v;
  return GS_OK;
}

// Tile-rasterisation group height (1..255; 0 = default 8) for tuning sweeps.
GS_KERNEL_API int gs_gemm_set_group_m(int g) {
  if (g < 0 || g > 255) return GS_EINVAL;
  g_group_m = g;
  return GS_OK;
}
