// Decode-phase GQA attention over a KV cache (split-K, "flash-decoding"), plus the KV append.
//
// Serving pods decode one token per sequence per step, so attention reads the whole KV cache
// once and does ~1 FLOP/byte: it is HBM-bound and the job is to stream K and V at full
// bandwidth with enough workgroups in flight. Layout and schedule:
//   * cache [B, Hkv, Smax, D=128] bf16: one (sequence, kv head) is a contiguous Smax x 256 B
//     slab, so a chunk of positions is one contiguous stream;
//   * grid (Smax / CHUNK, Hkv, B): a workgroup owns CHUNK = 256 positions of one (b, kv head)
//     and all G = Hq / Hkv query heads that share it (K/V read once per group, not per head);
//     workgroups past lens[b] exit at once, so the grid can be sized from the cache capacity
//     and the kernel needs no host-side length (it is captured in a hipGraph once and replayed);
//   * scores: 8 lanes per position, 16 dims (two 16-B loads) each, a wave covers 8 positions per
//     step and the 4 waves 32: 64 lanes x 32 B = 2 KiB contiguous per wave-step; q is pre-scaled
//     by softmax_scale * log2(e) so the softmax runs on exp2;
//   * softmax: one wave per query head, over the CHUNK scores held in LDS;
//   * P·V: each wave instruction reads 4 whole V rows (16 lanes x 16 B per row) and every lane
//     accumulates all G heads for its 8 dims; shuffles + an LDS pass reduce rows and waves
//     (the first version gave each head its own 16 lanes, so an instruction fetched one 256-B
//     row four times over: 2.85 TB/s in the model, profiles/decode/README.md);
//   * partials (m, l, unnormalised o) per split go to a float workspace; a second kernel merges
//     the splits of each (b, q head) and writes bf16.
#include "common.h"

namespace {

constexpr int D = 128;
constexpr int CHUNK = 256;
constexpr int NT = 256;
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// NTL: K and V rows are loaded non-temporal (the cache is streamed once per step).
template <int G, bool NTL = false>
__global__ __launch_bounds__(NT) void decode_split(const unsigned short* __restrict__ q, int q_bstride,
                                                   const unsigned short* __restrict__ kc,
                                                   const unsigned short* __restrict__ vc,
                                                   const int* __restrict__ lens, float* __restrict__ o_part,
                                                   float* __restrict__ ml_part, int Hkv, int Smax, int nsplit,
                                                   float qscale) {
  __shared__ float S[G][CHUNK];
  __shared__ float red[4][G * D];
  __shared__ float ML[G][2];

  const int kvh = blockIdx.x, b = blockIdx.y, split = blockIdx.z;   // chunks slowest: dead ones dispatch last
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int len = min(lens[b], Smax);
  const int c0 = split * CHUNK;
  const int Hq = Hkv * G;
  if (c0 >= len) return;                  // nothing here; the merge kernel never reads this split
  const int n = min(CHUNK, len - c0);

  const size_t slab = ((size_t)b * Hkv + kvh) * Smax;
  const unsigned short* kp = kc + (slab + c0) * D;
  const unsigned short* vp = vc + (slab + c0) * D;

  // ---- scores ---------------------------------------------------------------------------
  const int part = tid & 7;               // dims [16 part, 16 part + 16)
  float qf[G][16];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const unsigned short* qh = q + (size_t)b * q_bstride + (kvh * G + g) * D + part * 16;
    const u16x8_t q0 = *(const u16x8_t*)qh, q1 = *(const u16x8_t*)(qh + 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      qf[g][i] = bf16_to_f32(q0[i]) * qscale;
      qf[g][8 + i] = bf16_to_f32(q1[i]) * qscale;
    }
  }
#pragma unroll
  for (int step = 0; step < CHUNK / 32; ++step) {
    const int p = step * 32 + (tid >> 3);
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) s[g] = 0.f;
    if (p < n) {
      const unsigned short* kr = kp + (size_t)p * D + part * 16;
      u16x8_t k0, k1;
      if constexpr (NTL) {
        k0 = __builtin_nontemporal_load((const u16x8_t*)kr);
        k1 = __builtin_nontemporal_load((const u16x8_t*)(kr + 8));
      } else {
        k0 = *(const u16x8_t*)kr;
        k1 = *(const u16x8_t*)(kr + 8);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float a = bf16_to_f32(k0[i]), c = bf16_to_f32(k1[i]);
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] = fmaf(qf[g][i], a, fmaf(qf[g][8 + i], c, s[g]));
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float v = s[g];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      if (part == 0) S[g][p] = p < n ? v : -INFINITY;
    }
  }
  __syncthreads();

  // ---- softmax over the chunk: wave w handles heads w, w + 4, ... --------------------------
  for (int g = wave; g < G; g += 4) {
    float m = -INFINITY;
#pragma unroll
    for (int i = lane; i < CHUNK; i += 64) m = fmaxf(m, S[g][i]);
    m = wave_max(m);
    float l = 0.f;
#pragma unroll
    for (int i = lane; i < CHUNK; i += 64) {
      const float e = i < n ? exp2f(S[g][i] - m) : 0.f;
      S[g][i] = e;
      l += e;
    }
    l = wave_sum(l);
    if (lane == 0) {
      ML[g][0] = m;
      ML[g][1] = l;
    }
  }
  __syncthreads();

  // ---- P·V: lane -> (row r = lane / 16, dims (lane % 16) * 8); a wave instruction reads 4 whole
  // V rows (1 KiB) and every lane accumulates all G heads for its 8 dims; the 4 row lanes of a dim
  // group are then summed with two shuffles and the 4 waves through LDS ------------------------
  const int rsub = lane >> 4, d0 = (lane & 15) * 8;
  float acc[G][8];
#pragma unroll
  for (int gg = 0; gg < G; ++gg)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[gg][i] = 0.f;
#pragma unroll 8
  for (int p = wave * 4 + rsub; p < n; p += 16) {
    const u16x8_t* vsrc = (const u16x8_t*)(vp + (size_t)p * D + d0);
    u16x8_t v8;
    if constexpr (NTL)
      v8 = __builtin_nontemporal_load(vsrc);
    else
      v8 = *vsrc;
    float vf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) vf[i] = bf16_to_f32(v8[i]);
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      const float w = S[gg][p];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[gg][i] = fmaf(w, vf[i], acc[gg][i]);
    }
  }
#pragma unroll
  for (int gg = 0; gg < G; ++gg)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = acc[gg][i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      acc[gg][i] = v;
    }
  if (rsub == 0) {
#pragma unroll
    for (int gg = 0; gg < G; ++gg)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[wave][gg * D + d0 + i] = acc[gg][i];
  }
  __syncthreads();
  for (int e = tid; e < G * D; e += NT) {
    const int gg = e / D, d = e % D;
    const float o = red[0][e] + red[1][e] + red[2][e] + red[3][e];
    const size_t row = ((size_t)b * Hq + kvh * G + gg) * nsplit + split;
    o_part[row * D + d] = o;
    if (d == 0) {
      ml_part[row * 2] = ML[gg][0];
      ml_part[row * 2 + 1] = ML[gg][1];
    }
  }
}

__global__ __launch_bounds__(D) void decode_merge(const float* __restrict__ o_part, const float* __restrict__ ml_part,
                                                  const int* __restrict__ lens, unsigned short* __restrict__ out,
                                                  int Hq, int Smax, int nsplit) {
  // a latency kernel: lane s < ns fetches split s's (max, sum) pair, and every thread issues its o
  // loads 8 at a time before using them; the combine order (split 0, 1, ...) is unchanged
  __shared__ float2 MLs[D];
  const int hq = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int len = min(lens[b], Smax);
  const int ns = (len + CHUNK - 1) / CHUNK;
  const size_t row0 = ((size_t)b * Hq + hq) * nsplit;
  float m = -INFINITY;
  for (int s0 = 0; s0 < ns; s0 += D) {
    const int s = s0 + d;
    const float2 v = s < ns ? *(const float2*)(ml_part + (row0 + s) * 2) : make_float2(-INFINITY, 0.f);
    if (s0 == 0) MLs[d] = v;
    m = fmaxf(m, v.x);
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wmax[D / 64];
  if ((d & 63) == 0) wmax[d >> 6] = m;
  __syncthreads();
#pragma unroll
  for (int w = 0; w < D / 64; ++w) m = fmaxf(m, wmax[w]);
  float num = 0.f, den = 0.f;
  for (int s0 = 0; s0 < ns; s0 += 8) {
    float ov[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) ov[j] = s0 + j < ns ? o_part[(row0 + s0 + j) * D + d] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int s = s0 + j;
      if (s >= ns) break;
      const float2 ml = s < D ? MLs[s] : *(const float2*)(ml_part + (row0 + s) * 2);
      const float w = exp2f(ml.x - m);
      den = fmaf(w, ml.y, den);
      num = fmaf(w, ov[j], num);
    }
  }
  out[((size_t)b * Hq + hq) * D + d] = f32_to_bf16(den > 0.f ? num / den : 0.f);
}

// cache[b][h][pos[b]][:] = src[b][h * D : (h + 1) * D] for K and V; one 16-B chunk per thread.
__global__ __launch_bounds__(256) void kv_append(const unsigned short* __restrict__ k, const unsigned short* __restrict__ v,
                                                 int src_bstride, unsigned short* __restrict__ kc,
                                                 unsigned short* __restrict__ vc, const int* __restrict__ pos, int B,
                                                 int Hkv, int Smax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;      // over B * Hkv * (D / 8) * 2
  const int per = Hkv * (D / 8);
  if (i >= 2 * B * per) return;
  const int which = i / (B * per), r = i % (B * per);
  const int b = r / per, h = (r % per) / (D / 8), c = r % (D / 8);
  const int p = pos[b];
  if (p < 0 || p >= Smax) return;
  const unsigned short* src = (which ? v : k) + (size_t)b * src_bstride + h * D + c * 8;
  unsigned short* dst = (which ? vc : kc) + ((((size_t)b * Hkv + h) * Smax + p) * D) + c * 8;
  *(u16x8_t*)dst = *(const u16x8_t*)src;
}

// Decode-step fusion of RoPE(q), RoPE(k) and the KV append (one launch instead of three): per
// sequence b at position pos[b], q and k heads of the fused QKV row are rotated in place (4 pairs
// per thread, cos/sin from the host tables) and the rotated k plus the raw v are written to the
// caches. Items per sequence: (Hq + Hkv) heads x D/8 rotation items, then Hkv x D/8 v copies.
__global__ __launch_bounds__(256) void rope_kv_append(unsigned short* __restrict__ qkv, int bstride,
                                                      const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                      int tab_rows, const int* __restrict__ pos,
                                                      unsigned short* __restrict__ kc, unsigned short* __restrict__ vc,
                                                      int B, int Hq, int Hkv, int Smax) {
  constexpr int HALF = D / 2, NQ = HALF / 4;           // 16 rotation items per head
  constexpr int NV = D / 8;                            // 16 copy items per v head
  const int per = (Hq + Hkv) * NQ + Hkv * NV;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * per) return;
  const int b = i / per, r = i % per;
  const int p = pos[b];
  const bool in_cache = p >= 0 && p < Smax;
  unsigned short* row = qkv + (size_t)b * bstride;
  if (r < (Hq + Hkv) * NQ) {
    const int h = r / NQ, d = (r % NQ) * 4;
    const int pt = min(max(p, 0), tab_rows - 1);
    unsigned short* hp = row + (size_t)h * D;
    const u16x4_t a = *(const u16x4_t*)(hp + d);
    const u16x4_t c2 = *(const u16x4_t*)(hp + HALF + d);
    const float4 c = *(const float4*)(cosb + (size_t)pt * HALF + d);
    const float4 sn = *(const float4*)(sinb + (size_t)pt * HALF + d);
    const float cc[4] = {c.x, c.y, c.z, c.w}, sc[4] = {sn.x, sn.y, sn.z, sn.w};
    u16x4_t oa, ob;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x1 = bf16_to_f32(a[e]), x2 = bf16_to_f32(c2[e]);
      oa[e] = f32_to_bf16(x1 * cc[e] - x2 * sc[e]);
      ob[e] = f32_to_bf16(x2 * cc[e] + x1 * sc[e]);
    }
    *(u16x4_t*)(hp + d) = oa;
    *(u16x4_t*)(hp + HALF + d) = ob;
    if (h >= Hq && in_cache) {
      unsigned short* dst = kc + ((((size_t)b * Hkv + (h - Hq)) * Smax + p) * D);
      *(u16x4_t*)(dst + d) = oa;
      *(u16x4_t*)(dst + HALF + d) = ob;
    }
  } else if (in_cache) {
    const int r2 = r - (Hq + Hkv) * NQ, h = r2 / NV, c = (r2 % NV) * 8;
    const unsigned short* src = row + (size_t)(Hq + Hkv + h) * D + c;
    *(u16x8_t*)(vc + ((((size_t)b * Hkv + h) * Smax + p) * D) + c) = *(const u16x8_t*)src;
  }
}

}  // namespace

GS_KERNEL_API int gs_rope_kv_append_bf16(void* qkv, int bstride, const float* cosb, const float* sinb, int tab_rows,
                                         const int* pos, void* k_cache, void* v_cache, int B, int Hq, int Hkv, int Dh,
                                         int Smax, hipStream_t stream) {
  if (Dh != D || B <= 0 || Hq <= 0 || Hkv <= 0 || Smax <= 0 || tab_rows <= 0 || bstride % 8 ||
      bstride < (Hq + 2 * Hkv) * D)
    return GS_EINVAL;
  const int n = B * ((Hq + Hkv) * (D / 8) + Hkv * (D / 8));
  hipLaunchKernelGGL(rope_kv_append, dim3((n + 255) / 256), dim3(256), 0, stream, (unsigned short*)qkv, bstride, cosb,
                     sinb, tab_rows, pos, (unsigned short*)k_cache, (unsigned short*)v_cache, B, Hq, Hkv, Smax);
  return gs_launch_status();
}

// K/V load policy of the split kernel (0 plain, 1 non-temporal, the default): the cache is read once
// per step, so it is streamed non-temporal; 1.5-5 % faster with caches streamed from HBM and the
// batch-32 decode step 0.6 % (profiles/decode/decode_nt_r3_*.jsonl).
static int g_dec_nt = 1;

GS_KERNEL_API int gs_decode_attn_set_nt(int on) {
  if (on != 0 && on != 1) return GS_EINVAL;
  g_dec_nt = on;
  return GS_OK;
}

// q: [B, Hq, D] rows at q_bstride elements per sequence (heads contiguous); caches [B, Hkv, Smax, D];
// lens[B] (device); workspace: o_part [B, Hq, nsplit, D] f32 + ml_part [B, Hq, nsplit, 2] f32 with
// nsplit = ceil(Smax / 256); out [B, Hq, D] bf16.
GS_KERNEL_API int gs_decode_attn_bf16(const void* q, int q_bstride, const void* k_cache, const void* v_cache,
                                      const int* lens, void* o_part, void* ml_part, void* out, int B, int Hq, int Hkv,
                                      int Dh, int Smax, float scale, hipStream_t stream) {
  if (Dh != D || B <= 0 || Hkv <= 0 || Hq % Hkv || Smax <= 0 || Smax % CHUNK || q_bstride < Hq * D || q_bstride % 8)
    return GS_EINVAL;
  const int G = Hq / Hkv, nsplit = Smax / CHUNK;
  const dim3 grid(Hkv, B, nsplit);
  const float qs = scale * LOG2E;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(NT), 0, stream, (const unsigned short*)q, q_bstride,
                       (const unsigned short*)k_cache, (const unsigned short*)v_cache, lens, (float*)o_part,
                       (float*)ml_part, Hkv, Smax, nsplit, qs);
  };
  switch (G * 2 + (g_dec_nt ? 1 : 0)) {
    case 2: args(decode_split<1>); break;
    case 3: args(decode_split<1, true>); break;
    case 4: args(decode_split<2>); break;
    case 5: args(decode_split<2, true>); break;
    case 8: args(decode_split<4>); break;
    case 9: args(decode_split<4, true>); break;
    case 16: args(decode_split<8>); break;
    case 17: args(decode_split<8, true>); break;
    default: return GS_EINVAL;
  }
  hipLaunchKernelGGL(decode_merge, dim3(Hq, B), dim3(D), 0, stream, (const float*)o_part, (const float*)ml_part, lens,
                     (unsigned short*)out, Hq, Smax, nsplit);
  return gs_launch_status();
}

// k/v: [B, Hkv * D] rows at src_bstride elements (slices of the fused QKV output); pos[B] device.
GS_KERNEL_API int gs_kv_append_bf16(const void* k, const void* v, int src_bstride, void* k_cache, void* v_cache,
                                    const int* pos, int B, int Hkv, int Dh, int Smax, hipStream_t stream) {
  if (Dh != D || B <= 0 || Hkv <= 0 || Smax <= 0 || src_bstride < Hkv * D || src_bstride % 8) return GS_EINVAL;
  const int n = 2 * B * Hkv * (D / 8);
  hipLaunchKernelGGL(kv_append, dim3((n + 255) / 256), dim3(256), 0, stream, (const unsigned short*)k,
                     (const unsigned short*)v, src_bstride, (unsigned short*)k_cache, (unsigned short*)v_cache, pos, B,
                     Hkv, Smax);
  return gs_launch_status();
}
