// Transformer (BERT-base MLM, BASELINE.json config 5) kernels for gfx950: SURVEY.md N-K7/N-K8.
//
//  * LayerNorm forward/backward with the surrounding elementwise work fused in:
//      s = dropout(a + bias) + residual ;  y = dropout_post(LN(s))
//    (encoder sub-layers use the pre-dropout + residual form, the embeddings the post-dropout
//    form).  One wave per row, every lane owns NV 4-element chunks (H = 256*NV); backward
//    emits dx plus deterministic per-block partial sums of dgamma / dbeta / dbias that a
//    column-reduction kernel folds in fixed order (no atomics).
//  * bias + GELU (tanh form of google-research/bert modeling.py) forward / backward with the
//    bias gradient reduced in the same pass.
//  * Flash-style attention for head_dim 64 on v_mfma_f32_16x16x32_bf16, reading Q/K/V straight
//    out of the fused [T, 3*H*64] QKV GEMM output (no transposes) and writing [T, H*64]:
//      fwd  : per 16-query wave, S^T = K.Q^T so every lane owns ONE query column -> the online
//             softmax max/sum is lane-local except one xor-16/xor-32 exchange; P^T goes from the
//             accumulator straight into the B operand of O^T = V^T.P^T (keys permuted
//             consistently in both operands), V^T is read with ds_read_b64_tr_b16.
//      bwd  : two deterministic kernels (no dQ atomics): dK/dV per 16-key wave sweeping all
//             queries, dQ per 16-query wave sweeping all keys; P is recomputed from the saved
//             log2-domain LSE; delta = rowsum(dO*O) comes from a small prep kernel.
//    Attention dropout uses a counter-based hash of (seed, b, h, q, k) so the backward
//    regenerates the mask instead of storing it.
//  * Embedding gather+sum+LN forward, deterministic segment-sum backward for the word table.
//  * MLM cross-entropy over bf16 logits with per-prediction weights (loss = sum(w*nll)/sum(w)).
#include <type_traits>

#include "common.h"

namespace {

constexpr float kLog2e = 1.4426950408889634f;

DTF_DEV uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
// keep with probability 1 - thr/2^32 (thr == 0: dropout off)
DTF_DEV bool keep_elem(uint32_t seed, uint32_t idx, uint32_t thr) {
  return fmix32(idx * 0x9E3779B1u + seed) >= thr;
}

DTF_DEV void load4(const bf16_t* p, float* f) {
  const uint2 v = *(const uint2*)p;
  f[0] = __builtin_bit_cast(float, v.x << 16);
  f[1] = __builtin_bit_cast(float, v.x & 0xffff0000u);
  f[2] = __builtin_bit_cast(float, v.y << 16);
  f[3] = __builtin_bit_cast(float, v.y & 0xffff0000u);
}
DTF_DEV void store4(bf16_t* p, const float* f) {
  uint2 v;
  v.x = pack2(f[0], f[1]);
  v.y = pack2(f[2], f[3]);
  *(uint2*)p = v;
}
DTF_DEV float round_bf(float x) { return bf2f(f2bf(x)); }

struct LnArgs {
  const bf16_t* a;        // [M, H] main input
  const float* bias;      // [H] or null (added to a before the pre-dropout)
  const bf16_t* res;      // [M, H] or null
  const float* gamma;
  const float* beta;
  bf16_t* y;              // [M, H] output
  bf16_t* s;              // [M, H] saved LN input (null: not saved; then s == a)
  float* mean;
  float* rstd;
  // embedding mode (a == null): s = word[ids] + pos[row % S] + type[tt]
  const int64_t* ids;
  const int64_t* tt;
  const bf16_t* word;
  const bf16_t* pos;
  const bf16_t* type;
  int M, S;
  float eps;
  uint32_t seed_pre, thr_pre;
  uint32_t seed_post, thr_post;
  float inv_keep_pre, inv_keep_post;
};

template <int NV>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const LnArgs g) {
  constexpr int H = NV * 256;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= g.M) return;
  const long base = (long)row * H;
  float v[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (g.a) {
      load4(g.a + base + col, v[i]);
      if (g.bias) {   // one 16-B load for the 4 columns (was 4 scalar loads)
        const float4 b4 = *reinterpret_cast<const float4*>(g.bias + col);
        v[i][0] += b4.x; v[i][1] += b4.y; v[i][2] += b4.z; v[i][3] += b4.w;
      }
      if (g.thr_pre) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[i][e] = keep_elem(g.seed_pre, (uint32_t)(base + col + e), g.thr_pre)
                        ? v[i][e] * g.inv_keep_pre : 0.f;
      }
      if (g.res) {
        float r[4];
        load4(g.res + base + col, r);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[i][e] += r[e];
      }
    } else {
      float w[4], p[4], t[4];
      load4(g.word + g.ids[row] * (long)H + col, w);
      load4(g.pos + (long)(row % g.S) * H + col, p);
      load4(g.type + (g.tt ? g.tt[row] : 0) * (long)H + col, t);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i][e] = w[e] + p[e] + t[e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[i][e] = round_bf(v[i][e]);   // stats of exactly what is saved
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) sum += v[i][e];
  const float mean = wave_sum(sum) * (1.f / H);
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      sq += d * d;
    }
  const float rstd = rsqrtf(wave_sum(sq) * (1.f / H) + g.eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (g.s) store4(g.s + base + col, v[i]);
    float o[4];
    const float4 g4 = *reinterpret_cast<const float4*>(g.gamma + col);
    const float4 be4 = *reinterpret_cast<const float4*>(g.beta + col);
    const float gm[4] = {g4.x, g4.y, g4.z, g4.w}, bt[4] = {be4.x, be4.y, be4.z, be4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = (v[i][e] - mean) * rstd * gm[e] + bt[e];
      if (g.thr_post)
        o[e] = keep_elem(g.seed_post, (uint32_t)(base + col + e), g.thr_post)
                   ? o[e] * g.inv_keep_post : 0.f;
    }
    store4(g.y + base + col, o);
  }
  if (lane == 0) {
    g.mean[row] = mean;
    g.rstd[row] = rstd;
  }
}

struct LnBwdArgs {
  const bf16_t* dy;       // [M, H]
  const bf16_t* s;        // saved LN input
  const float* mean;
  const float* rstd;
  const float* gamma;
  bf16_t* ds;             // [M, H] d(LN input) (= d residual)
  bf16_t* da;             // [M, H] d(a) when a pre-dropout was applied (else null: da == ds)
  float* part_g;          // [nblk, H]
  float* part_b;          // [nblk, H]
  float* part_bias;       // [nblk, H] or null
  int M, rows_per_block;
  uint32_t seed_pre, thr_pre, seed_post, thr_post;
  float inv_keep_pre, inv_keep_post;
};

template <int NV>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const LnBwdArgs g) {
  constexpr int H = NV * 256;
  __shared__ float red[4][H];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ag[NV][4], ab[NV][4], abias[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) ag[i][e] = ab[i][e] = abias[i][e] = 0.f;
  const int r0 = blockIdx.x * g.rows_per_block;
  const int r1 = min(g.M, r0 + g.rows_per_block);
  float gm[NV][4];           // gamma of this lane's columns, loaded once (not per row)
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float4 g4 = *reinterpret_cast<const float4*>(g.gamma + (i * 64 + lane) * 4);
    gm[i][0] = g4.x; gm[i][1] = g4.y; gm[i][2] = g4.z; gm[i][3] = g4.w;
  }
  for (int row = r0 + wave; row < r1; row += 4) {
    const long base = (long)row * H;
    const float mean = g.mean[row], rstd = g.rstd[row];
    float dy[NV][4], xh[NV][4], gy[NV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * 64 + lane) * 4;
      float sv[4];
      load4(g.dy + base + col, dy[i]);
      load4(g.s + base + col, sv);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (g.thr_post)
          dy[i][e] = keep_elem(g.seed_post, (uint32_t)(base + col + e), g.thr_post)
                         ? dy[i][e] * g.inv_keep_post : 0.f;
        xh[i][e] = (sv[e] - mean) * rstd;
        gy[i][e] = dy[i][e] * gm[i][e];
        s1 += gy[i][e];
        s2 += gy[i][e] * xh[i][e];
      }
    }
    s1 = wave_sum(s1) * (1.f / H);
    s2 = wave_sum(s2) * (1.f / H);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = (i * 64 + lane) * 4;
      float dx[4], da[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dx[e] = rstd * (gy[i][e] - s1 - xh[i][e] * s2);
        ag[i][e] += dy[i][e] * xh[i][e];
        ab[i][e] += dy[i][e];
        if (g.thr_pre)
          da[e] = keep_elem(g.seed_pre, (uint32_t)(base + col + e), g.thr_pre)
                      ? dx[e] * g.inv_keep_pre : 0.f;
        else
          da[e] = dx[e];
        abias[i][e] += da[e];
      }
      store4(g.ds + base + col, dx);
      if (g.da) store4(g.da + base + col, da);
    }
  }
  // fixed-order block reduction of the three column partials
  float* outs[3] = {g.part_g, g.part_b, g.part_bias};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (!outs[k]) continue;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        red[wave][(i * 64 + lane) * 4 + e] = k == 0 ? ag[i][e] : (k == 1 ? ab[i][e] : abias[i][e]);
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += 256)
      outs[k][(long)blockIdx.x * H + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  }
}

// 16-B variants ("wide"): a HALF wave per row, every lane moving 16-B chunks (8 elements) at
// columns (c * 32 + lane) * 8 -- the 8-B-per-lane kernels above read / wrote ~70 % of the HBM rate
// at BERT's H = 768.  Same per-element arithmetic and dropout indices; the row statistics are the
// same sums in a different lane order.
DTF_DEV float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}
DTF_DEV void load8b(const bf16_t* p, float* f) { unpack8(*reinterpret_cast<const uint4*>(p), f); }
DTF_DEV void store8b(bf16_t* p, const float* f) { *reinterpret_cast<uint4*>(p) = pack8(f); }

template <int NC>
__global__ void __launch_bounds__(256) ln_fwd_wide_kernel(const LnArgs g) {
  constexpr int H = NC * 256;
  const int hl = threadIdx.x & 31;
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (row >= g.M) return;           // whole half-waves: the shuffles stay inside a half
  const long base = (long)row * H;
  float v[NC][8];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int col = (i * 32 + hl) * 8;
    if (g.a) {
      load8b(g.a + base + col, v[i]);
      if (g.bias) {
        const float4 b0 = *reinterpret_cast<const float4*>(g.bias + col);
        const float4 b1 = *reinterpret_cast<const float4*>(g.bias + col + 4);
        v[i][0] += b0.x; v[i][1] += b0.y; v[i][2] += b0.z; v[i][3] += b0.w;
        v[i][4] += b1.x; v[i][5] += b1.y; v[i][6] += b1.z; v[i][7] += b1.w;
      }
      if (g.thr_pre) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[i][e] = keep_elem(g.seed_pre, (uint32_t)(base + col + e), g.thr_pre)
                        ? v[i][e] * g.inv_keep_pre : 0.f;
      }
      if (g.res) {
        float r[8];
        load8b(g.res + base + col, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] += r[e];
      }
    } else {
      float w[8], p[8], t[8];
      load8b(g.word + g.ids[row] * (long)H + col, w);
      load8b(g.pos + (long)(row % g.S) * H + col, p);
      load8b(g.type + (g.tt ? g.tt[row] : 0) * (long)H + col, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = w[e] + p[e] + t[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[i][e] = round_bf(v[i][e]);
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += v[i][e];
  const float mean = half_sum(sum) * (1.f / H);
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[i][e] - mean;
      sq += d * d;
    }
  const float rstd = rsqrtf(half_sum(sq) * (1.f / H) + g.eps);
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int col = (i * 32 + hl) * 8;
    if (g.s) store8b(g.s + base + col, v[i]);
    float o[8];
    const float4 g0 = *reinterpret_cast<const float4*>(g.gamma + col);
    const float4 g1 = *reinterpret_cast<const float4*>(g.gamma + col + 4);
    const float4 e0 = *reinterpret_cast<const float4*>(g.beta + col);
    const float4 e1 = *reinterpret_cast<const float4*>(g.beta + col + 4);
    const float gm[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bt[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = (v[i][e] - mean) * rstd * gm[e] + bt[e];
      if (g.thr_post)
        o[e] = keep_elem(g.seed_post, (uint32_t)(base + col + e), g.thr_post)
                   ? o[e] * g.inv_keep_post : 0.f;
    }
    store8b(g.y + base + col, o);
  }
  if (hl == 0) {
    g.mean[row] = mean;
    g.rstd[row] = rstd;
  }
}

template <int NC>
__global__ void __launch_bounds__(256) ln_bwd_wide_kernel(const LnBwdArgs g) {
  constexpr int H = NC * 256;
  __shared__ float red[8][H];
  const int hl = threadIdx.x & 31, half = threadIdx.x >> 5;
  float ag[NC][8], ab[NC][8], abias[NC][8];
#pragma unroll
  for (int i = 0; i < NC; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) ag[i][e] = ab[i][e] = abias[i][e] = 0.f;
  const int r0 = blockIdx.x * g.rows_per_block;
  const int r1 = min(g.M, r0 + g.rows_per_block);
  for (int row = r0 + half; row < r1; row += 8) {
    const long base = (long)row * H;
    const float mean = g.mean[row], rstd = g.rstd[row];
    float xh[NC][8], gy[NC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int col = (i * 32 + hl) * 8;
      float sv[8], dy[8];
      load8b(g.dy + base + col, dy);
      load8b(g.s + base + col, sv);
      const float4 g0 = *reinterpret_cast<const float4*>(g.gamma + col);
      const float4 g1 = *reinterpret_cast<const float4*>(g.gamma + col + 4);
      const float gm[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (g.thr_post)
          dy[e] = keep_elem(g.seed_post, (uint32_t)(base + col + e), g.thr_post)
                      ? dy[e] * g.inv_keep_post : 0.f;
        xh[i][e] = (sv[e] - mean) * rstd;
        gy[i][e] = dy[e] * gm[e];
        ag[i][e] += dy[e] * xh[i][e];
        ab[i][e] += dy[e];
        s1 += gy[i][e];
        s2 += gy[i][e] * xh[i][e];
      }
    }
    s1 = half_sum(s1) * (1.f / H);
    s2 = half_sum(s2) * (1.f / H);
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int col = (i * 32 + hl) * 8;
      float dx[8], da[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dx[e] = rstd * (gy[i][e] - s1 - xh[i][e] * s2);
        if (g.thr_pre)
          da[e] = keep_elem(g.seed_pre, (uint32_t)(base + col + e), g.thr_pre)
                      ? dx[e] * g.inv_keep_pre : 0.f;
        else
          da[e] = dx[e];
        abias[i][e] += da[e];
      }
      store8b(g.ds + base + col, dx);
      if (g.da) store8b(g.da + base + col, da);
    }
  }
  float* outs[3] = {g.part_g, g.part_b, g.part_bias};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (!outs[k]) continue;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NC; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        red[half][(i * 32 + hl) * 8 + e] = k == 0 ? ag[i][e] : (k == 1 ? ab[i][e] : abias[i][e]);
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += 256) {
      float t = 0.f;
#pragma unroll
      for (int h2 = 0; h2 < 8; ++h2) t += red[h2][c];
      outs[k][(long)blockIdx.x * H + c] = t;
    }
  }
}

// out[c] (+)= sum_p part[p, c] in fixed order
// Deterministic two-level column sum of a [P][N] fp32 partial slab (N % 4 == 0):
//   level 1: grid (N/256 float4-column groups, S row slices); 4 waves = 4 row groups, each lane
//            one float4 column, fixed-order LDS combine -> ws[S][N]
//   level 2: one thread per float4 column sums the S slices in order.
// (A single pass of one thread per column serialised 512 dependent loads on 3 blocks: 130 us
// per LayerNorm backward at BERT-base shape, 30 % of the step.)
constexpr int kColSplits = 32;
struct ColSumOut { float* p[3]; };

// blockIdx.z = quantity q: its partial rows start at part + q * region, its level-1 workspace
// right after them (P rows in)
__global__ void __launch_bounds__(256)
col_sum_split_kernel(const float* __restrict__ part, long region, int P, int N, int R) {
  __shared__ float4 red[4][64];
  const float* pq = part + blockIdx.z * region;
  float* ws = const_cast<float*>(pq) + (long)P * N;
  const int c4 = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * R;
  const int r1 = min(P, r0 + R);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 * 4 < N) {
#pragma unroll 4
    for (int r = r0 + rg; r < r1; r += 4) {
      const float4 v = reinterpret_cast<const float4*>(pq + (long)r * N)[c4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c4 * 4 < N) {
    float4 t = red[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 v = red[k][threadIdx.x];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    reinterpret_cast<float4*>(ws + (long)blockIdx.y * N)[c4] = t;
  }
}

// level 2: 64 float4 columns x 4 slice groups per block, fixed-order combine
__global__ void __launch_bounds__(256)
col_sum_final_kernel(const float* __restrict__ part, long region, int P, int S, int N, ColSumOut outs,
                     int accumulate) {
  __shared__ float4 red[4][64];
  const float* ws = part + blockIdx.z * region + (long)P * N;
  const int c4 = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 * 4 < N)
    for (int k = rg; k < S; k += 4) {
      const float4 v = reinterpret_cast<const float4*>(ws + (long)k * N)[c4];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
  red[rg][threadIdx.x & 63] = t;
  __syncthreads();
  if (rg == 0 && c4 * 4 < N) {
    float4 u = red[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 v = red[k][threadIdx.x];
      u.x += v.x; u.y += v.y; u.z += v.z; u.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(outs.p[blockIdx.z]) + c4;
    if (accumulate) { const float4 v = *o; u.x += v.x; u.y += v.y; u.z += v.z; u.w += v.w; }
    *o = u;
  }
}

// part: nq quantities, each `region` floats apart: [P][N] partial rows then kColSplits rows of
// workspace.  Two launches regardless of nq.
void col_sum(const float* part, long region, int nq, int P, int N, ColSumOut outs, hipStream_t st,
             int accumulate = 0) {
  int S = P / 16;
  S = S < 1 ? 1 : (S > kColSplits ? kColSplits : S);
  const int R = (P + S - 1) / S;
  const int gx = (N / 4 + 63) / 64;
  hipLaunchKernelGGL(col_sum_split_kernel, dim3(gx, S, nq), dim3(256), 0, st, part, region, P, N, R);
  hipLaunchKernelGGL(col_sum_final_kernel, dim3(gx, 1, nq), dim3(256), 0, st, part, region, P, S, N, outs,
                     accumulate);
}

// Column sums of a bf16 [T][N] matrix into fp32 (bias gradients of library-GEMM dense layers):
// level 1 reads 16 B (8 columns) per lane, 4 row groups per block, 4 rows in flight per lane,
// grid (N/512, S slices of R rows) -> ws[S][N]; level 2 (bf16_col_sum_final_kernel) sums the S
// slices in a fixed order with 16 row groups per 16 float4 columns, so even N = 768 spreads over
// enough blocks (the first version used 32 slices: 64 blocks for N = 768, ~0.4 TB/s).
constexpr int kBf16ColSplits = 256;

// VEC bf16 columns per lane: 8 (16-B loads; N % 8 == 0) or 2 (4-B loads; any even N, e.g. the
// 30522-wide MLM decoder bias)
template <int VEC>
__global__ void __launch_bounds__(256)
bf16_col_sum_split_kernel(const bf16_t* __restrict__ x, int T, int N, float* __restrict__ ws, int R) {
  __shared__ float red[4][64][VEC + 1];
  const int cv = blockIdx.x * 64 + (threadIdx.x & 63);      // VEC-column vector index
  const int rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * R, r1 = min(T, r0 + R);
  float acc[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
  typedef typename std::conditional<VEC == 8, uint4, uint32_t>::type vec_t;
  auto add = [&](const vec_t& v) {
    if constexpr (VEC == 8) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += f[e];
    } else {
      acc[0] += __builtin_bit_cast(float, v << 16);
      acc[1] += __builtin_bit_cast(float, v & 0xffff0000u);
    }
  };
  if (cv * VEC < N) {
    const vec_t* X4 = reinterpret_cast<const vec_t*>(x) + cv;
    const long rs = N / VEC;
    int r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      vec_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = X4[(long)(r + 4 * u) * rs];
#pragma unroll
      for (int u = 0; u < 4; ++u) add(v[u]);
    }
    for (; r < r1; r += 4) add(X4[(long)r * rs]);
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) red[rg][threadIdx.x & 63][e] = acc[e];
  __syncthreads();
  if (rg == 0 && cv * VEC < N) {
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      float t = red[0][threadIdx.x][e];
#pragma unroll
      for (int k = 1; k < 4; ++k) t += red[k][threadIdx.x][e];
      ws[(long)blockIdx.y * N + cv * VEC + e] = t;
    }
  }
}

// level 2: 16 column vectors (float4, or single floats when N % 4 != 0) x 16 slice groups per
// block, fixed-order combine (+= into out)
template <int W>
__global__ void __launch_bounds__(256)
bf16_col_sum_final_kernel(const float* __restrict__ ws, int S, int N, float* __restrict__ out,
                          int accumulate) {
  __shared__ float red[16][16][W];
  const int c4 = blockIdx.x * 16 + (threadIdx.x & 15);
  const int rg = threadIdx.x >> 4;
  float t[W];
#pragma unroll
  for (int e = 0; e < W; ++e) t[e] = 0.f;
  if (c4 * W < N)
    for (int k = rg; k < S; k += 16) {
      if constexpr (W == 4) {
        const float4 v = reinterpret_cast<const float4*>(ws + (long)k * N)[c4];
        t[0] += v.x; t[1] += v.y; t[2] += v.z; t[3] += v.w;
      } else {
        t[0] += ws[(long)k * N + c4];
      }
    }
#pragma unroll
  for (int e = 0; e < W; ++e) red[rg][threadIdx.x & 15][e] = t[e];
  __syncthreads();
  if (rg == 0 && c4 * W < N) {
    float u[W];
#pragma unroll
    for (int e = 0; e < W; ++e) {
      u[e] = red[0][threadIdx.x][e];
#pragma unroll
      for (int k = 1; k < 16; ++k) u[e] += red[k][threadIdx.x][e];
      if (accumulate) u[e] += out[c4 * W + e];
      out[c4 * W + e] = u[e];
    }
  }
}

}  // namespace

int dtf_bf16_col_sum_ws_floats(int N) { return kBf16ColSplits * N; }

void dtf_bf16_col_sum(const bf16_t* x, int T, int N, float* ws, float* out, int accumulate,
                      hipStream_t st) {
  if (N % 2) throw std::runtime_error("bf16_col_sum: N % 2 != 0");
  int S = T / 64;
  S = S < 1 ? 1 : (S > kBf16ColSplits ? kBf16ColSplits : S);
  const int R = (T + S - 1) / S;
  if (N % 8 == 0)
    hipLaunchKernelGGL(bf16_col_sum_split_kernel<8>, dim3((N / 8 + 63) / 64, S), dim3(256), 0, st,
                       x, T, N, ws, R);
  else
    hipLaunchKernelGGL(bf16_col_sum_split_kernel<2>, dim3((N / 2 + 63) / 64, S), dim3(256), 0, st,
                       x, T, N, ws, R);
  if (N % 4 == 0)
    hipLaunchKernelGGL(bf16_col_sum_final_kernel<4>, dim3((N / 4 + 15) / 16), dim3(256), 0, st,
                       ws, S, N, out, accumulate);
  else
    hipLaunchKernelGGL(bf16_col_sum_final_kernel<1>, dim3((N + 15) / 16), dim3(256), 0, st, ws, S,
                       N, out, accumulate);
}

namespace {

// ----------------------------------------------------------------------------- bias + GELU
// GELU (tanh form) and its derivative: common.h (shared with the GEMM's GELU-backward epilogue)

// Row sweep (as bias_gelu_bwd_kernel): block = R rows x all columns, a thread owns column vectors
// cv = tid + 256 j with the bias in registers and keeps 4 rows' 16-B loads in flight (the r1
// one-vector-per-thread form did a 32-bit modulo and 8 scalar bias loads per vector and ran at
// ~2.3 TB/s on the BERT FFN activation).
__global__ void __launch_bounds__(256)
bias_gelu_fwd_kernel(const bf16_t* __restrict__ a, const float* __restrict__ bias,
                     bf16_t* __restrict__ y, int M, int N, int R) {
  constexpr int U = 4;
  const int nv = N / 8;
  const int r0 = blockIdx.x * R, r1 = min(M, r0 + R);
  const uint4* A4 = reinterpret_cast<const uint4*>(a);
  uint4* Y4 = reinterpret_cast<uint4*>(y);
  for (int cv = threadIdx.x; cv < nv; cv += 256) {
    float bb[8];
    if (bias) {
      const float4 b0 = reinterpret_cast<const float4*>(bias)[cv * 2];
      const float4 b1 = reinterpret_cast<const float4*>(bias)[cv * 2 + 1];
      bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
      bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bb[e] = 0.f;
    }
    for (int r = r0; r < r1; r += U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (r + u < r1) v[u] = A4[(uint32_t)(r + u) * nv + cv];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + u >= r1) break;
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = gelu_f(f[e] + bb[e]);
        Y4[(uint32_t)(r + u) * nv + cv] = pack8(f);
      }
    }
  }
}

// block = (row tile of R rows) x (all columns); thread owns column vectors cv = tid + 256*j
__global__ void __launch_bounds__(256)
bias_gelu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ a,
                     const float* __restrict__ bias, bf16_t* __restrict__ da,
                     float* __restrict__ part, int M, int N, int R) {
  const int nv = N / 8;
  const int r0 = blockIdx.x * R, r1 = min(M, r0 + R);
  for (int cv = threadIdx.x; cv < nv; cv += 256) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float bb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bb[e] = bias ? bias[cv * 8 + e] : 0.f;
    for (int r = r0; r < r1; ++r) {
      const long off = (long)r * nv + cv;
      float fd[8], fa[8];
      unpack8(((const uint4*)dy)[off], fd);
      unpack8(((const uint4*)a)[off], fa);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        fd[e] *= gelu_grad(fa[e] + bb[e]);
        acc[e] += fd[e];
      }
      ((uint4*)da)[off] = pack8(fd);
    }
    if (part) {
#pragma unroll
      for (int e = 0; e < 8; ++e) part[(long)blockIdx.x * N + cv * 8 + e] = acc[e];
    }
  }
}

// ----------------------------------------------------------------------------- attention
constexpr int AD = 64;    // head dim
constexpr int ALD = 72;   // LDS row pitch in elements (144 B: 16-B aligned rows, spread banks)

typedef __attribute__((ext_vector_type(4))) short s4_t;
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

struct AttnGeom {
  int B, S, H, ld;        // ld = row pitch of the qkv / dqkv buffers (3*H*64)
  float scale;            // softmax scale (1/sqrt(64))
  uint32_t seed, thr;     // attention-probability dropout
  float inv_keep;
  // S == 128 with dropout (8-wave forward + fused backward): the forward's keep decisions, one
  // 32-bit word per (b, h, query, 16-lane group) -- bit 4 t + r = key 16 t + 4 group + r, the
  // keys of exactly that lane in both kernels -- so the backward reads 4 B instead of 32 hashes
  uint32_t* keep;
};

DTF_DEV bf16x8_t lds_row8(const bf16_t* base, int row, int col) {
  return *(const bf16x8_t*)(base + row * ALD + col);
}
// 8 keys x one column for an MFMA operand whose k index is the key permutation
//   j < 4 : key row0 + 4g + j,   j >= 4 : key row0 + 16 + 4g + (j - 4)
// read with ds_read_b64_tr_b16 (lane 4q+p of each 16-lane group addresses row q, cols 4p..4p+3)
DTF_DEV bf16x8_t lds_tr8(const bf16_t* base, int row0, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const bf16_t* p = base + (row0 + 4 * g + (i >> 2)) * ALD + col0 + 4 * (i & 3);
  const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(p));
  const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(p + 16 * ALD));
  return (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
DTF_DEV bf16x8_t pack_frag(const f32x4_t& x0, const f32x4_t& x1) {
  return (bf16x8_t){(short)f2bf(x0[0]), (short)f2bf(x0[1]), (short)f2bf(x0[2]), (short)f2bf(x0[3]),
                    (short)f2bf(x1[0]), (short)f2bf(x1[1]), (short)f2bf(x1[2]), (short)f2bf(x1[3])};
}
DTF_DEV f32x4_t mfma(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// Explicit wait states between an MFMA chain and the first VALU / accvgpr read of its result.
// Measured need: with a (uniform) branch between the last MFMA and the read, hipcc's hazard
// recognizer only padded the fall-through path, and the taken path read the accumulator ~1
// instruction after a 16x16x32 MFMA issued (wrong dQ whenever dropout was off).  Fencing the
// scheduler on both sides keeps every consumer behind the nops.
DTF_DEV void mfma_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
DTF_DEV void store4_scaled(bf16_t* p, const f32x4_t& v, float s) {
  const float f[4] = {v[0] * s, v[1] * s, v[2] * s, v[3] * s};
  store4(p, f);
}

// cooperative CH-row x 64-col loads of two operands (NT threads, 16 B per chunk)
template <int NT, int CH>
DTF_DEV void load_two_tiles(bf16_t* d0, const bf16_t* s0, long ld0, bf16_t* d1, const bf16_t* s1,
                            long ld1, int tid) {
  constexpr int kChunks = 2 * CH * 8;
  static_assert(kChunks % NT == 0, "tile chunks must divide over the block");
#pragma unroll
  for (int i = 0; i < kChunks / NT; ++i) {
    const int v = tid + NT * i;
    const int sel = v / (CH * 8), row = (v >> 3) % CH, cc = (v & 7) * 8;
    const uint4 x = sel ? *(const uint4*)(s1 + row * ld1 + cc) : *(const uint4*)(s0 + row * ld0 + cc);
    *(uint4*)((sel ? d1 : d0) + row * ALD + cc) = x;
  }
}

// Launch shapes: NW waves x 16 rows per block, K/V (or Q/dO) staged CH rows at a time.  <8, 128>
// (S % 128 == 0, e.g. BERT's 128) covers a whole 128-token sequence per block, so each (b, h)
// reads its K/V once instead of once per 64-query block and syncs once per 128 keys.
template <bool DROP, int NW, int CH>
__global__ void __launch_bounds__(64 * NW)
attn_fwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                bf16_t* __restrict__ out, float* __restrict__ lse, const AttnGeom g) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[CH * ALD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[CH * ALD];
  __shared__ float Ms[CH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, gq = lane >> 4, li = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z, S = g.S, H = g.H;
  const long tok0 = (long)b * S;
  const int q = blockIdx.x * 16 * NW + w * 16 + li;
  const bf16_t* qrow = qkv + (tok0 + q) * g.ld + h * AD;
  const bf16x8_t bq0 = *(const bf16x8_t*)(qrow + 8 * gq);
  const bf16x8_t bq1 = *(const bf16x8_t*)(qrow + 32 + 8 * gq);
  const float c = g.scale * kLog2e;
  const uint32_t kbase = (uint32_t)((((long)b * H + h) * S + q) * S);
  float m = -INFINITY, l = 0.f;
  uint32_t kbits = 0;                    // keep decisions (S == CH == 128: one key chunk)
  f32x4_t acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  for (int kc = 0; kc < S; kc += CH) {
    __syncthreads();
    load_two_tiles<64 * NW, CH>(Ks, qkv + (tok0 + kc) * g.ld + (H + h) * AD, g.ld,
                                Vs, qkv + (tok0 + kc) * g.ld + (2 * H + h) * AD, g.ld, tid);
    if (tid < CH) Ms[tid] = mask ? mask[tok0 + kc + tid] * kLog2e : 0.f;
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < CH; sub += 64) {
      const bf16_t* Kb = Ks + sub * ALD;
      const bf16_t* Vb = Vs + sub * ALD;
      f32x4_t s[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        s[t] = mfma(lds_row8(Kb, 16 * t + li, 8 * gq), bq0, s[t]);
        s[t] = mfma(lds_row8(Kb, 16 * t + li, 32 + 8 * gq), bq1, s[t]);
      }
      mfma_fence();
      float mloc = -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[t][r] = s[t][r] * c + Ms[sub + 16 * t + 4 * gq + r];
          mloc = fmaxf(mloc, s[t][r]);
        }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float mnew = fmaxf(m, mloc);
      const float alpha = exp2f(m - mnew);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] *= alpha;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[t][r] - mnew);
          l += p;
          if (DROP) {
            const bool kp = keep_elem(g.seed, kbase + kc + sub + 16 * t + 4 * gq + r, g.thr);
            s[t][r] = kp ? p * g.inv_keep : 0.f;
            if constexpr (CH == 128) kbits |= (uint32_t)kp << ((sub >> 6) * 16 + 4 * t + r);
          } else {
            s[t][r] = p;
          }
        }
      const bf16x8_t bp0 = pack_frag(s[0], s[1]);
      const bf16x8_t bp1 = pack_frag(s[2], s[3]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        acc[dt] = mfma(lds_tr8(Vb, 0, 16 * dt, lane), bp0, acc[dt]);
        acc[dt] = mfma(lds_tr8(Vb, 32, 16 * dt, lane), bp1, acc[dt]);
      }
      m = mnew;
    }
  }
  mfma_fence();
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  bf16_t* orow = out + (tok0 + q) * (long)(H * AD) + h * AD;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) store4_scaled(orow + 16 * dt + 4 * gq, acc[dt], inv);
  if (gq == 0) lse[((long)b * H + h) * S + q] = m + log2f(l);
  if constexpr (DROP && CH == 128)
    if (g.keep) g.keep[(((long)b * H + h) * S + q) * 4 + gq] = kbits;
}

template <bool DROP, int NW, int CH>
__global__ void __launch_bounds__(64 * NW)
attn_bwd_dkv_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                    const bf16_t* __restrict__ dO, const float* __restrict__ lse,
                    const float* __restrict__ delta, bf16_t* __restrict__ dqkv, const AttnGeom g) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[CH * ALD];
  __shared__ __attribute__((aligned(16))) bf16_t Os[CH * ALD];
  __shared__ float Ls[CH], Ds[CH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, gq = lane >> 4, li = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z, S = g.S, H = g.H;
  const long tok0 = (long)b * S;
  const int k = blockIdx.x * 16 * NW + w * 16 + li;       // this lane's key
  const bf16_t* krow = qkv + (tok0 + k) * g.ld + (H + h) * AD;
  const bf16_t* vrow = qkv + (tok0 + k) * g.ld + (2 * H + h) * AD;
  const bf16x8_t bk0 = *(const bf16x8_t*)(krow + 8 * gq), bk1 = *(const bf16x8_t*)(krow + 32 + 8 * gq);
  const bf16x8_t bv0 = *(const bf16x8_t*)(vrow + 8 * gq), bv1 = *(const bf16x8_t*)(vrow + 32 + 8 * gq);
  const float mk = mask ? mask[tok0 + k] * kLog2e : 0.f;
  const float c = g.scale * kLog2e;
  const long bh = (long)b * H + h;
  f32x4_t dv[4], dk[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dv[dt] = dk[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  for (int qc = 0; qc < S; qc += CH) {
    __syncthreads();
    load_two_tiles<64 * NW, CH>(Qs, qkv + (tok0 + qc) * g.ld + h * AD, g.ld,
                                Os, dO + (tok0 + qc) * (long)(H * AD) + h * AD, H * AD, tid);
    if (tid < CH) {
      Ls[tid] = lse[bh * S + qc + tid];
      Ds[tid] = delta[bh * S + qc + tid];
    }
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < CH; sub += 64) {
      const bf16_t* Qb = Qs + sub * ALD;
      const bf16_t* Ob = Os + sub * ALD;
      f32x4_t P[4], dS[4];
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        f32x4_t s = (f32x4_t){0.f, 0.f, 0.f, 0.f}, dp = s;
        s = mfma(lds_row8(Qb, 16 * qt + li, 8 * gq), bk0, s);
        s = mfma(lds_row8(Qb, 16 * qt + li, 32 + 8 * gq), bk1, s);
        dp = mfma(lds_row8(Ob, 16 * qt + li, 8 * gq), bv0, dp);
        dp = mfma(lds_row8(Ob, 16 * qt + li, 32 + 8 * gq), bv1, dp);
        mfma_fence();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = sub + 16 * qt + 4 * gq + r;
          const float p = exp2f(s[r] * c + mk - Ls[qq]);
          if (DROP) {
            const bool kp = keep_elem(g.seed, (uint32_t)((bh * S + qc + qq) * S + k), g.thr);
            P[qt][r] = kp ? p * g.inv_keep : 0.f;
            dS[qt][r] = p * ((kp ? dp[r] * g.inv_keep : 0.f) - Ds[qq]);
          } else {
            P[qt][r] = p;
            dS[qt][r] = p * (dp[r] - Ds[qq]);
          }
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t bP = pack_frag(P[2 * ks], P[2 * ks + 1]);
        const bf16x8_t bS = pack_frag(dS[2 * ks], dS[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          dv[dt] = mfma(lds_tr8(Ob, 32 * ks, 16 * dt, lane), bP, dv[dt]);
          dk[dt] = mfma(lds_tr8(Qb, 32 * ks, 16 * dt, lane), bS, dk[dt]);
        }
      }
    }
  }
  // dV^T / dK^T accumulators: column = this lane's key, rows d = 16dt + 4gq + r
  mfma_fence();
  bf16_t* dkrow = dqkv + (tok0 + k) * g.ld + (H + h) * AD;
  bf16_t* dvrow = dqkv + (tok0 + k) * g.ld + (2 * H + h) * AD;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    store4_scaled(dkrow + 16 * dt + 4 * gq, dk[dt], g.scale);
    store4_scaled(dvrow + 16 * dt + 4 * gq, dv[dt], 1.f);
  }
}

template <bool DROP, int NW, int CH>
__global__ void __launch_bounds__(64 * NW)
attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                   const bf16_t* __restrict__ dO, const float* __restrict__ lse,
                   float* __restrict__ delta, bf16_t* __restrict__ dqkv, const AttnGeom g,
                   const bf16_t* __restrict__ O) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[CH * ALD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[CH * ALD];
  __shared__ float Ms[CH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, gq = lane >> 4, li = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z, S = g.S, H = g.H;
  const long tok0 = (long)b * S;
  const int q = blockIdx.x * 16 * NW + w * 16 + li;
  const bf16_t* qrow = qkv + (tok0 + q) * g.ld + h * AD;
  const bf16_t* orow = dO + (tok0 + q) * (long)(H * AD) + h * AD;
  const bf16x8_t bq0 = *(const bf16x8_t*)(qrow + 8 * gq), bq1 = *(const bf16x8_t*)(qrow + 32 + 8 * gq);
  const bf16x8_t bo0 = *(const bf16x8_t*)(orow + 8 * gq), bo1 = *(const bf16x8_t*)(orow + 32 + 8 * gq);
  const long bh = (long)b * H + h;
  const float lq = lse[bh * S + q];
  // delta = O . dO of this lane's query: the 4 lane groups hold 16 of its 64 columns each; the
  // dK/dV kernel (launched after this one) reads it back
  float dl;
  {
    const bf16_t* oq = O + (tok0 + q) * (long)(H * AD) + h * AD;
    const uint4 o0 = *(const uint4*)(oq + 8 * gq), o1 = *(const uint4*)(oq + 32 + 8 * gq);
    float fo[8], fd[8];
    dl = 0.f;
    unpack8(o0, fo);
    unpack8(*(const uint4*)(orow + 8 * gq), fd);
#pragma unroll
    for (int e = 0; e < 8; ++e) dl += fo[e] * fd[e];
    unpack8(o1, fo);
    unpack8(*(const uint4*)(orow + 32 + 8 * gq), fd);
#pragma unroll
    for (int e = 0; e < 8; ++e) dl += fo[e] * fd[e];
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    if (gq == 0) delta[bh * S + q] = dl;
  }
  const float c = g.scale * kLog2e;
  const uint32_t kbase = (uint32_t)((bh * S + q) * S);
  f32x4_t dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  for (int kc = 0; kc < S; kc += CH) {
    __syncthreads();
    load_two_tiles<64 * NW, CH>(Ks, qkv + (tok0 + kc) * g.ld + (H + h) * AD, g.ld,
                                Vs, qkv + (tok0 + kc) * g.ld + (2 * H + h) * AD, g.ld, tid);
    if (tid < CH) Ms[tid] = mask ? mask[tok0 + kc + tid] * kLog2e : 0.f;
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < CH; sub += 64) {
      const bf16_t* Kb = Ks + sub * ALD;
      const bf16_t* Vb = Vs + sub * ALD;
      f32x4_t dS[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x4_t s = (f32x4_t){0.f, 0.f, 0.f, 0.f}, dp = s;
        s = mfma(lds_row8(Kb, 16 * t + li, 8 * gq), bq0, s);
        s = mfma(lds_row8(Kb, 16 * t + li, 32 + 8 * gq), bq1, s);
        dp = mfma(lds_row8(Vb, 16 * t + li, 8 * gq), bo0, dp);
        dp = mfma(lds_row8(Vb, 16 * t + li, 32 + 8 * gq), bo1, dp);
        mfma_fence();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = sub + 16 * t + 4 * gq + r;
          const float p = exp2f(s[r] * c + Ms[key] - lq);
          float dpu = dp[r];
          if (DROP) dpu = keep_elem(g.seed, kbase + kc + key, g.thr) ? dpu * g.inv_keep : 0.f;
          dS[t][r] = p * (dpu - dl);
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8_t bS = pack_frag(dS[2 * ks], dS[2 * ks + 1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma(lds_tr8(Kb, 32 * ks, 16 * dt, lane), bS, dq[dt]);
      }
    }
  }
  mfma_fence();
  bf16_t* dqrow = dqkv + (tok0 + q) * g.ld + h * AD;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) store4_scaled(dqrow + 16 * dt + 4 * gq, dq[dt], g.scale);
}

// Fused backward for S == 128 (BERT-base at seq 128): ONE 8-wave block per (b, h) holds the whole
// sequence -- Q, K, V and dO staged once in LDS -- and forms dQ, dK and dV in two phases:
//   1. wave w, queries 16w..16w+15 (the dQ kernel's work over all 128 keys): S = Q K^T and
//      dP = dO V^T per 16-key group, P = exp(S - lse) (+ dropout), dS = P (dP - delta),
//      dQ = dS K; P (dropped) and dS are kept, rounded to bf16 exactly as the split kernels'
//      fragments round them;
//   2. wave w takes keys 16w..16w+15, reading [query][key] tiles in LDS with the same
//      transposing ds_read_b64_tr_b16 fragments the dK/dV kernel builds in registers: P goes over
//      the dead K|V region and dV = P^T dO; then dS over the same region and dK = dS^T Q.
// Against dQ + dK/dV as two kernels this drops the second Q K^T and dO V^T (5 instead of 7
// 128 x 128 x 64 products per (b, h)) and the second read of Q / K / V / dO; every accumulator
// sums in the same order as before, so the gradients are bit-identical to the split kernels.
// P and dS taking turns in one region keeps the block at 80 KB of LDS and <= 128 VGPRs: TWO
// blocks per CU, so one block's Q/K/V/dO loads overlap the other's MFMAs (one block per CU left
// the matrix pipe idle for the whole load phase).
constexpr int kFusedS = 128, kPLD = 136;   // P / dS row pitch (272 B: 8-B aligned rows)
constexpr int kFusedRed = 8 * 3 * AD;        // [wave][dq | dk | dv column] fp32 partial sums
constexpr int kFusedLds = (4 * kFusedS * ALD) * 2 + kFusedS * 4 + kFusedRed * 4;   // 80,384 B

// sum of v over the 16 lanes of this lane's 16-lane group (the 16 queries / keys of a wave)
DTF_DEV float sum16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

DTF_DEV bf16x8_t lds_tr8_p(const bf16_t* base, int row0, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const bf16_t* p = base + (row0 + 4 * g + (i >> 2)) * kPLD + col0 + 4 * (i & 3);
  const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(p));
  const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(p + 16 * kPLD));
  return (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// One (b, h) pair's backward from its staged LDS image (Q, K, V, dO rows at pitch ALD, the key
// mask).  ``orow``: this lane's 16 B of O at columns 8 gq and 32 + 8 gq of its query row
// (delta = O . dO with dO from the staged image: 2 global loads per lane fewer than re-reading
// it, 4-8 % off the kernel).  (A persistent form -- one block per CU, the next pair's rows
// prefetched into registers under the current pair -- measured 1.5x SLOWER: one block per CU
// leaves the pair's dependent MFMA / exp chain exposed that two co-resident blocks interleave.)
template <bool DROP>
DTF_DEV void attn_bwd_pair(bf16_t* fsm, int b, int h, const float* __restrict__ lse,
                           float* __restrict__ delta, bf16_t* __restrict__ dqkv, const AttnGeom& g,
                           const uint4 (&orow)[2], float* __restrict__ colpart) {
  constexpr int S = kFusedS;
  bf16_t* Qs = fsm;
  bf16_t* Os = Qs + S * ALD;                 // dO
  bf16_t* KV = Os + S * ALD;                 // K | V, then P, then dS
  bf16_t* dSs = KV;
  float* Ms = reinterpret_cast<float*>(KV + 2 * S * ALD);
  float* red = Ms + S;                       // [8 waves][3 * 64] column partials (colpart)
  bf16_t* Ks = KV;
  bf16_t* Vs = KV + S * ALD;
  bf16_t* Ps = KV;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, gq = lane >> 4, li = lane & 15;
  const int H = g.H;
  const long tok0 = (long)b * S, bh = (long)b * H + h;
  // ---- this lane's query q: lse and delta = O . dO (dO from the staged image: the same bits)
  const int q = w * 16 + li;
  const float lq = lse[bh * S + q];
  float dl = 0.f;
  {
    float fo[8], fd[8];
    unpack8(orow[0], fo);
    unpack8(*(const uint4*)(Os + q * ALD + 8 * gq), fd);
#pragma unroll
    for (int e = 0; e < 8; ++e) dl += fo[e] * fd[e];
    unpack8(orow[1], fo);
    unpack8(*(const uint4*)(Os + q * ALD + 32 + 8 * gq), fd);
#pragma unroll
    for (int e = 0; e < 8; ++e) dl += fo[e] * fd[e];
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    if (gq == 0) delta[bh * S + q] = dl;
  }
  // ---- phase 1: this wave's 16 queries against all 128 keys
  const bf16x8_t bq0 = lds_row8(Qs, q, 8 * gq), bq1 = lds_row8(Qs, q, 32 + 8 * gq);
  const bf16x8_t bo0 = lds_row8(Os, q, 8 * gq), bo1 = lds_row8(Os, q, 32 + 8 * gq);
  const float c = g.scale * kLog2e;
  const uint32_t kbase = (uint32_t)((bh * S + q) * S);
  const uint32_t kw = (DROP && g.keep) ? g.keep[(bh * S + q) * 4 + gq] : 0u;
  // P and dS are only ever used rounded to bf16 (MFMA fragments, LDS tiles): kept packed, 4 keys
  // per uint2 -- half the registers of fp32, same bits
  uint2 P[8], dS[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4_t s = (f32x4_t){0.f, 0.f, 0.f, 0.f}, dp = s;
    float pt[4], st[4];
    s = mfma(lds_row8(Ks, 16 * t + li, 8 * gq), bq0, s);
    s = mfma(lds_row8(Ks, 16 * t + li, 32 + 8 * gq), bq1, s);
    dp = mfma(lds_row8(Vs, 16 * t + li, 8 * gq), bo0, dp);
    dp = mfma(lds_row8(Vs, 16 * t + li, 32 + 8 * gq), bo1, dp);
    mfma_fence();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * t + 4 * gq + r;
      const float p = exp2f(s[r] * c + Ms[key] - lq);
      if (DROP) {
        const bool kp = g.keep ? ((kw >> (4 * t + r)) & 1u) != 0u : keep_elem(g.seed, kbase + key, g.thr);
        pt[r] = kp ? p * g.inv_keep : 0.f;
        st[r] = p * ((kp ? dp[r] * g.inv_keep : 0.f) - dl);
      } else {
        pt[r] = p;
        st[r] = p * (dp[r] - dl);
      }
    }
    P[t] = make_uint2(pack2(pt[0], pt[1]), pack2(pt[2], pt[3]));
    dS[t] = make_uint2(pack2(st[0], st[1]), pack2(st[2], st[3]));
  }
  f32x4_t acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8_t bS = __builtin_bit_cast(
        bf16x8_t, make_uint4(dS[2 * ks].x, dS[2 * ks].y, dS[2 * ks + 1].x, dS[2 * ks + 1].y));
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] = mfma(lds_tr8(Ks, 32 * ks, 16 * dt, lane), bS, acc[dt]);
  }
  mfma_fence();
  {
    bf16_t* dqrow = dqkv + (tok0 + q) * g.ld + h * AD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) store4_scaled(dqrow + 16 * dt + 4 * gq, acc[dt], g.scale);
    if (colpart) {
      // column sums of the STORED (bf16-rounded) dQ over this wave's 16 queries
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t = sum16(round_bf(acc[dt][r] * g.scale));
          if (li == 0) red[w * 3 * AD + 16 * dt + 4 * gq + r] = t;
        }
    }
  }
  __syncthreads();                 // every wave is done with K and V: P may overwrite them
  // ---- [query][key] tiles: this lane's 4 consecutive keys of each group
  auto put = [&](bf16_t* dst, const uint2 (&v)[8]) {
#pragma unroll
    for (int t = 0; t < 8; ++t) *(uint2*)(dst + q * kPLD + 16 * t + 4 * gq) = v[t];
  };
  put(Ps, P);
  __syncthreads();
  // ---- phase 2: this wave's 16 keys against all 128 queries; dV from P first
  const int k = w * 16 + li;
  f32x4_t dv[4], dk[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dv[dt] = dk[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8_t bP = lds_tr8_p(Ps, 32 * ks, 16 * w, lane);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dv[dt] = mfma(lds_tr8(Os, 32 * ks, 16 * dt, lane), bP, dv[dt]);
  }
  mfma_fence();
  bf16_t* dkrow = dqkv + (tok0 + k) * g.ld + (H + h) * AD;
  bf16_t* dvrow = dqkv + (tok0 + k) * g.ld + (2 * H + h) * AD;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) store4_scaled(dvrow + 16 * dt + 4 * gq, dv[dt], 1.f);
  if (colpart) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float tv = sum16(round_bf(dv[dt][r]));
        if (li == 0) red[w * 3 * AD + 2 * AD + 16 * dt + 4 * gq + r] = tv;
      }
  }
  __syncthreads();                 // every wave is done reading P: dS takes its place
  put(dSs, dS);
  __syncthreads();
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8_t bS = lds_tr8_p(dSs, 32 * ks, 16 * w, lane);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[dt] = mfma(lds_tr8(Qs, 32 * ks, 16 * dt, lane), bS, dk[dt]);
  }
  mfma_fence();
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) store4_scaled(dkrow + 16 * dt + 4 * gq, dk[dt], g.scale);
  if (colpart) {
    // the qkv bias gradient's first level: per (b, h) column sums of dQ / dK / dV over the 128
    // tokens (8 waves x 16, fixed order) -> colpart[b][3 * H * 64], in dqkv's column layout;
    // the _Dense backward of the QKV projection sums the B rows instead of re-reading dqkv
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float tk = sum16(round_bf(dk[dt][r] * g.scale));
        if (li == 0) red[w * 3 * AD + AD + 16 * dt + 4 * gq + r] = tk;
      }
    __syncthreads();
    if (tid < 3 * AD) {
      float t = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) t += red[ww * 3 * AD + tid];
      const int sec = tid / AD, col = tid % AD;
      colpart[(long)b * g.ld + (sec * H + h) * AD + col] = t;
    }
  }
}

// the pair's Q, K, V, dO rows (4 x 1024 16-B chunks over 512 threads): global -> registers ...
DTF_DEV void attn_bwd_pair_load(uint4 (&v)[8], float& mk, uint4 (&orow)[2], const bf16_t* qkv,
                                const float* mask, const bf16_t* dO, const bf16_t* O,
                                const AttnGeom& g, int b, int h) {
  constexpr int S = kFusedS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, gq = lane >> 4, li = lane & 15;
  const int H = g.H;
  const long tok0 = (long)b * S;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = tid + 512 * i;
    const int sel = c >> 10, row = (c >> 3) & (S - 1), cc = (c & 7) * 8;
    const bf16_t* src = sel == 3 ? dO + (tok0 + row) * (long)(H * AD) + h * AD + cc
                                 : qkv + (tok0 + row) * g.ld + (sel * H + h) * AD + cc;
    v[i] = *(const uint4*)src;
  }
  mk = (tid < S && mask) ? mask[tok0 + tid] * kLog2e : 0.f;
  const int q = w * 16 + li;
  const bf16_t* oq = O + (tok0 + q) * (long)(H * AD) + h * AD;
  orow[0] = *(const uint4*)(oq + 8 * gq);
  orow[1] = *(const uint4*)(oq + 32 + 8 * gq);
}
// ... -> the LDS image
DTF_DEV void attn_bwd_pair_store(bf16_t* fsm, const uint4 (&v)[8], float mk) {
  constexpr int S = kFusedS;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = tid + 512 * i;
    const int sel = c >> 10, row = (c >> 3) & (S - 1), cc = (c & 7) * 8;
    const int slot = sel == 0 ? 0 : sel == 3 ? 1 : sel + 1;       // image order Q | dO | K | V
    *(uint4*)(fsm + slot * S * ALD + row * ALD + cc) = v[i];
  }
  if (tid < S) reinterpret_cast<float*>(fsm + 4 * S * ALD)[tid] = mk;
}

template <bool DROP>
__global__ void __launch_bounds__(512, 4)      // 4 waves per SIMD = two 8-wave blocks per CU
attn_bwd_fused128_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                         const bf16_t* __restrict__ dO, const float* __restrict__ lse,
                         float* __restrict__ delta, bf16_t* __restrict__ dqkv, const AttnGeom g,
                         const bf16_t* __restrict__ O, float* __restrict__ colpart) {
  static_assert(kFusedS * kPLD <= 2 * kFusedS * ALD, "P / dS must fit over the K|V region");
  extern __shared__ __attribute__((aligned(16))) bf16_t fsm[];    // kFusedLds bytes (dynamic)
  const int h = blockIdx.x, b = blockIdx.y;
  uint4 v[8], orow[2];
  float mk;
  attn_bwd_pair_load(v, mk, orow, qkv, mask, dO, O, g, b, h);
  attn_bwd_pair_store(fsm, v, mk);
  __syncthreads();
  attn_bwd_pair<DROP>(fsm, b, h, lse, delta, dqkv, g, orow, colpart);
}

// ----------------------------------------------------------------------------- embeddings
// out[ids_sorted[i]] = sum over the run of equal ids of src[perm[j]]  (one wave per run start)
__global__ void __launch_bounds__(256)
segment_sum_kernel(const int64_t* __restrict__ sorted_ids, const int64_t* __restrict__ perm,
                   const bf16_t* __restrict__ src, float* __restrict__ out, int T, int H) {
  const int i = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= T) return;
  const int64_t id = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == id) return;
  for (int c0 = lane * 4; c0 < H; c0 += 256) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = i; j < T && sorted_ids[j] == id; ++j) {
      float v[4];
      load4(src + perm[j] * (long)H + c0, v);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += v[e];
    }
    float* o = out + id * (long)H + c0;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] += acc[e];
  }
}

// ----------------------------------------------------------------------------- MLM loss
// rows: loss_rows[i] = w_i * (lse - logit[label]) / denom ; grad = w_i * (softmax - onehot) / denom
// One wave per masked position.  Rows are `ld` elements apart (ld >= V): the tied MLM decoder runs
// on a vocabulary padded to a multiple of 64 (30528 for BERT's 30522), whose last ld - V logits
// are not classes -- they are left out of the softmax and their gradient is written as exact 0.
// With ld == V (rows only 4-B aligned) the row is swept in 16-B chunks from the 16-B-aligned
// address below its start with raw buffer loads (range-checked: the chunk before row 0 / past the
// last row reads zeros), elements outside the row masked.
// Online (max, sum) with one rescale per 8 elements; the gradient pass stores whole 16-B chunks
// inside the row and single elements at its two ends.
__global__ void __launch_bounds__(256)
mlm_xent_kernel(const bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                const float* __restrict__ weights, const float* __restrict__ denom, int N, int V,
                int ld, float* __restrict__ loss_rows, bf16_t* __restrict__ grad) {
  const int row = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const auto rl = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(logits), (short)0,
                                                    (int)((uint32_t)N * ld * 2u), 0x00020000);
  const uint32_t b0 = (uint32_t)row * ld * 2u;
  const uint32_t a0 = b0 & ~15u;
  const int head = (int)(b0 - a0) >> 1;
  const int nch = (head + V + 7) >> 3;
  float mx = -INFINITY, s = 0.f;
  for (int c = lane; c < nch; c += 64) {
    const uint4 raw = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rl, a0 + c * 16u, 0, 0));
    float f[8];
    unpack8(raw, f);
    const int e0 = c * 8 - head;
    float m8 = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (e0 + k < 0 || e0 + k >= V) f[k] = -INFINITY;
      m8 = fmaxf(m8, f[k]);
    }
    const float nm = fmaxf(mx, m8);
    float acc = mx == -INFINITY ? 0.f : s * __expf(mx - nm);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += __expf(f[k] - nm);   // exp(-inf) = 0 for masked slots
    s = acc;
    mx = nm;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(mx, om);
    s = (mx == -INFINITY ? 0.f : s * __expf(mx - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    mx = nm;
  }
  const float lse = mx + __logf(s);
  const int lab = (int)labels[row];
  const bf16_t* x = logits + (long)row * ld;
  const float wsc = weights ? weights[row] / fmaxf(denom[0], 1e-5f) : 1.f / fmaxf(denom[0], 1e-5f);
  if (lane == 0) loss_rows[row] = wsc * (lse - bf2f(x[lab]));
  if (grad) {
    // the whole stored row [0, ld): classes get the gradient, padding columns exact zeros
    const int gch = (head + ld + 7) >> 3;
    bf16_t* gbase = reinterpret_cast<bf16_t*>(reinterpret_cast<char*>(grad) + a0);
    for (int c = lane; c < gch; c += 64) {
      const uint4 raw = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rl, a0 + c * 16u, 0, 0));
      float f[8];
      unpack8(raw, f);
      const int e0 = c * 8 - head;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        f[k] = e0 + k < V ? wsc * (__expf(f[k] - lse) - (e0 + k == lab ? 1.f : 0.f)) : 0.f;
      if (e0 >= 0 && e0 + 8 <= ld) {
        reinterpret_cast<uint4*>(gbase)[c] = pack8(f);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (e0 + k >= 0 && e0 + k < ld) gbase[c * 8 + k] = f2bf(f[k]);
      }
    }
  }
}

}  // namespace

// ============================================================================= launchers

static uint32_t drop_thr(float p) {
  if (p <= 0.f) return 0u;
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 4294967295u : (uint32_t)t;
}

// 16-B half-wave-per-row LayerNorm kernels: bit 0 forward, bit 1 backward (the backward's 72
// per-lane column accumulators push it to ~190 VGPRs at H = 768: off unless measured faster)
static int g_ln_wide = 1;
void dtf_ln_set_wide(int v) { g_ln_wide = v; }

void dtf_ln_fwd(const bf16_t* a, const float* bias, const bf16_t* res, const float* gamma,
                const float* beta, bf16_t* y, bf16_t* s, float* mean, float* rstd, int M, int H,
                float eps, float p_pre, uint32_t seed_pre, float p_post, uint32_t seed_post,
                const int64_t* ids, const int64_t* tt, const bf16_t* word, const bf16_t* pos,
                const bf16_t* type, int S, hipStream_t st) {
  if (H % 256 != 0 || H > 1024) throw std::runtime_error("ln_fwd: H must be 256/512/768/1024");
  LnArgs g{a, bias, res, gamma, beta, y, s, mean, rstd, ids, tt, word, pos, type, M, S, eps,
           seed_pre, drop_thr(p_pre), seed_post, drop_thr(p_post),
           p_pre > 0.f ? 1.f / (1.f - p_pre) : 1.f, p_post > 0.f ? 1.f / (1.f - p_post) : 1.f};
  if (g_ln_wide & 1) {
    const dim3 gw((M + 7) / 8), bw(256);
    switch (H / 256) {
      case 1: hipLaunchKernelGGL(ln_fwd_wide_kernel<1>, gw, bw, 0, st, g); break;
      case 2: hipLaunchKernelGGL(ln_fwd_wide_kernel<2>, gw, bw, 0, st, g); break;
      case 3: hipLaunchKernelGGL(ln_fwd_wide_kernel<3>, gw, bw, 0, st, g); break;
      default: hipLaunchKernelGGL(ln_fwd_wide_kernel<4>, gw, bw, 0, st, g); break;
    }
    return;
  }
  const dim3 grid((M + 3) / 4), block(256);
  switch (H / 256) {
    case 1: hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, block, 0, st, g); break;
    case 2: hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, block, 0, st, g); break;
    case 3: hipLaunchKernelGGL(ln_fwd_kernel<3>, grid, block, 0, st, g); break;
    default: hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, block, 0, st, g); break;
  }
}

static int ln_bwd_rows(int M) { return (M + 31) / 32; }
// partial rows per reduced quantity, INCLUDING the column-sum workspace rows (allocation size)
int dtf_ln_bwd_blocks(int M) { return ln_bwd_rows(M) + kColSplits; }

void dtf_ln_bwd(const bf16_t* dy, const bf16_t* s, const float* mean, const float* rstd,
                const float* gamma, bf16_t* ds, bf16_t* da, float* part, float* dgamma,
                float* dbeta, float* dbias, int M, int H, float p_pre, uint32_t seed_pre,
                float p_post, uint32_t seed_post, hipStream_t st, int accumulate) {
  if (H % 256 != 0 || H > 1024) throw std::runtime_error("ln_bwd: H must be 256/512/768/1024");
  const int nblk = ln_bwd_rows(M);
  const long region = (long)dtf_ln_bwd_blocks(M) * H;   // partial rows + col-sum workspace
  float* pg = part;
  float* pb = part + region;
  float* pbias = dbias ? part + 2 * region : nullptr;
  LnBwdArgs g{dy, s, mean, rstd, gamma, ds, da, pg, pb, pbias, M, 32,
              seed_pre, drop_thr(p_pre), seed_post, drop_thr(p_post),
              p_pre > 0.f ? 1.f / (1.f - p_pre) : 1.f, p_post > 0.f ? 1.f / (1.f - p_post) : 1.f};
  const dim3 grid(nblk), block(256);
  if (g_ln_wide & 2) {
    switch (H / 256) {
      case 1: hipLaunchKernelGGL(ln_bwd_wide_kernel<1>, grid, block, 0, st, g); break;
      case 2: hipLaunchKernelGGL(ln_bwd_wide_kernel<2>, grid, block, 0, st, g); break;
      case 3: hipLaunchKernelGGL(ln_bwd_wide_kernel<3>, grid, block, 0, st, g); break;
      default: hipLaunchKernelGGL(ln_bwd_wide_kernel<4>, grid, block, 0, st, g); break;
    }
  } else {
    switch (H / 256) {
      case 1: hipLaunchKernelGGL(ln_bwd_kernel<1>, grid, block, 0, st, g); break;
      case 2: hipLaunchKernelGGL(ln_bwd_kernel<2>, grid, block, 0, st, g); break;
      case 3: hipLaunchKernelGGL(ln_bwd_kernel<3>, grid, block, 0, st, g); break;
      default: hipLaunchKernelGGL(ln_bwd_kernel<4>, grid, block, 0, st, g); break;
    }
  }
  col_sum(part, region, dbias ? 3 : 2, nblk, H, ColSumOut{{dgamma, dbeta, dbias}}, st, accumulate);
}

void dtf_bias_gelu_fwd(const bf16_t* a, const float* bias, bf16_t* y, long M, int N,
                       hipStream_t st) {
  if (N % 8) throw std::runtime_error("bias_gelu: N % 8 != 0");
  const long n8 = M * N / 8;
  if (n8 >= 2147483647L) throw std::runtime_error("bias_gelu: tensor too large");
  // ~1-2 blocks per CU-slot: R rows each (R a multiple of the 4-row unroll)
  int R = (int)((M + 2047) / 2048);
  R = ((R + 3) / 4) * 4;
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, dim3((unsigned)((M + R - 1) / R)), dim3(256), 0, st,
                     a, bias, y, (int)M, N, R);
}

static int bias_gelu_rows(int M) { return (M + 15) / 16; }
int dtf_bias_gelu_bwd_blocks(int M) { return bias_gelu_rows(M) + kColSplits; }

void dtf_bias_gelu_bwd(const bf16_t* dy, const bf16_t* a, const float* bias, bf16_t* da,
                       float* part, float* dbias, int M, int N, hipStream_t st, int accumulate) {
  if (N % 8) throw std::runtime_error("bias_gelu: N % 8 != 0");
  const int nblk = bias_gelu_rows(M);
  hipLaunchKernelGGL(bias_gelu_bwd_kernel, dim3(nblk), dim3(256), 0, st, dy, a, bias, da,
                     dbias ? part : nullptr, M, N, 16);
  if (dbias) col_sum(part, 0, 1, nblk, N, ColSumOut{{dbias, nullptr, nullptr}}, st, accumulate);
}

static AttnGeom attn_geom(int B, int S, int H, float scale, float p, uint32_t seed) {
  if (S % 64) throw std::runtime_error("attention: seq_len must be a multiple of 64");
  if ((long)B * H * S * S > 0xFFFFFFFFL && p > 0.f)
    throw std::runtime_error("attention dropout index space exceeds 32 bits");
  return AttnGeom{B, S, H, 3 * H * AD, scale, seed, drop_thr(p), p > 0.f ? 1.f / (1.f - p) : 1.f,
                  nullptr};
}

// 0: always the 4-wave / 64-row shape; 1 (default): 8 waves / 128 rows when S % 128 == 0
static int g_attn_wide = 1;
void dtf_attn_set_wide(int v) { g_attn_wide = v; }

// (the 8-wave forward takes 120 VGPRs: two blocks per CU; forcing 6 or 8 waves per SIMD spills
// and is 13-39 % slower with dropout, profiles/measurements/r4_attention_fwd_occupancy.jsonl)
template <int NW, int CH>
static void attn_fwd_launch(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse,
                            const AttnGeom& g, hipStream_t st) {
  const dim3 grid(g.S / (16 * NW), g.H, g.B);
  if (g.thr)
    hipLaunchKernelGGL((attn_fwd_kernel<true, NW, CH>), grid, dim3(64 * NW), 0, st, qkv, mask,
                       out, lse, g);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<false, NW, CH>), grid, dim3(64 * NW), 0, st, qkv, mask,
                       out, lse, g);
}

// dK/dV always runs the 4-wave shape: its 8-wave build needs 167 VGPRs with dropout (one block
// per CU) and measured 8 % slower on BERT-base; dQ gains 10 % from the 8-wave shape.
template <int NW, int CH>
static void attn_bwd_launch(const bf16_t* qkv, const float* mask, const bf16_t* out,
                            const bf16_t* dout, const float* lse, float* delta, bf16_t* dqkv,
                            const AttnGeom& g, hipStream_t st) {
  // dQ first: it also forms delta = O . dO per query (the separate delta pass is gone), which
  // the dK/dV kernel then reads
  const dim3 grid(g.S / (16 * NW), g.H, g.B), grid4(g.S / 64, g.H, g.B);
  if (g.thr) {
    hipLaunchKernelGGL((attn_bwd_dq_kernel<true, NW, CH>), grid, dim3(64 * NW), 0, st, qkv, mask,
                       dout, lse, delta, dqkv, g, out);
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<true, 4, 64>), grid4, dim3(256), 0, st, qkv, mask,
                       dout, lse, delta, dqkv, g);
  } else {
    hipLaunchKernelGGL((attn_bwd_dq_kernel<false, NW, CH>), grid, dim3(64 * NW), 0, st, qkv,
                       mask, dout, lse, delta, dqkv, g, out);
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<false, 4, 64>), grid4, dim3(256), 0, st, qkv, mask,
                       dout, lse, delta, dqkv, g);
  }
}

// 1 (default): with dropout at S == 128, the forward stores its keep decisions for the fused
// backward (dtf_attn_keep_words > 0)
static int g_attn_keep = 1;
void dtf_attn_set_keep(int v) { g_attn_keep = v; }
static int g_attn_fused = 1;
// uint32 words of the keep-decision buffer dtf_attn_fwd / dtf_attn_bwd take (0: not used)
long dtf_attn_keep_words(int B, int S, int H, float p) {
  return (g_attn_keep && g_attn_wide && g_attn_fused && S == 128 && p > 0.f) ? (long)B * H * S * 4
                                                                              : 0;
}

void dtf_attn_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse, int B, int S,
                  int H, float scale, float p, uint32_t seed, hipStream_t st, uint32_t* keep) {
  AttnGeom g = attn_geom(B, S, H, scale, p, seed);
  if (keep && !dtf_attn_keep_words(B, S, H, p))
    throw std::runtime_error("attn_fwd: keep buffer given for a shape that does not use it");
  g.keep = keep;
  if (g_attn_wide && S % 128 == 0) attn_fwd_launch<8, 128>(qkv, mask, out, lse, g, st);
  else attn_fwd_launch<4, 64>(qkv, mask, out, lse, g, st);
}

// 1 (default): S == 128 runs the fused one-block-per-(b, h) backward
void dtf_attn_set_fused(int v) { g_attn_fused = v; }

// 1 when dtf_attn_bwd will run the fused kernel for this shape (it can then also emit the qkv
// bias gradient's column partials)
int dtf_attn_bwd_fused(int S) { return g_attn_fused && S == kFusedS; }

void dtf_attn_bwd(const bf16_t* qkv, const float* mask, const bf16_t* out, const bf16_t* dout,
                  const float* lse, float* delta, bf16_t* dqkv, int B, int S, int H, float scale,
                  float p, uint32_t seed, hipStream_t st, float* colpart,
                  const uint32_t* keep) {
  AttnGeom g = attn_geom(B, S, H, scale, p, seed);
  if (colpart && !(g_attn_fused && S == kFusedS))
    throw std::runtime_error("attn_bwd: column partials need the fused S == 128 backward");
  if (keep && !dtf_attn_keep_words(B, S, H, p))
    throw std::runtime_error("attn_bwd: keep buffer given for a shape that does not use it");
  g.keep = const_cast<uint32_t*>(keep);
  if (g_attn_fused && S == kFusedS) {
    static bool attr = false;
    if (!attr) {
      HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_fused128_kernel<true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kFusedLds));
      HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_fused128_kernel<false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kFusedLds));
      attr = true;
    }
    const dim3 grid(H, B);
    if (g.thr)
      hipLaunchKernelGGL(attn_bwd_fused128_kernel<true>, grid, dim3(512), kFusedLds, st, qkv,
                         mask, dout, lse, delta, dqkv, g, out, colpart);
    else
      hipLaunchKernelGGL(attn_bwd_fused128_kernel<false>, grid, dim3(512), kFusedLds, st, qkv,
                         mask, dout, lse, delta, dqkv, g, out, colpart);
    return;
  }
  if (g_attn_wide && S % 128 == 0)
    attn_bwd_launch<8, 128>(qkv, mask, out, dout, lse, delta, dqkv, g, st);
  else
    attn_bwd_launch<4, 64>(qkv, mask, out, dout, lse, delta, dqkv, g, st);
}

namespace {

// Position- and token-type-embedding gradients of the embedding LayerNorm's output gradient ds
// [B*S][H] (bf16): dpos[s] = sum_b ds[b*S + s], dtyp[t] = sum of the rows whose type id is t.
// Level 1: block (s, 512-column chunk), 4 row groups x 64 lanes x 8 columns; the per-position
// type partials go to ws[s][t][H]; level 2 sums ws over s in a fixed order (deterministic; was a
// one-hot GEMM with N = 2 plus a bf16 -> fp32 copy and a reduction).
constexpr int kPosTypeMaxTypes = 4;

__global__ void __launch_bounds__(256)
pos_type_grad_kernel(const bf16_t* __restrict__ ds, const int64_t* __restrict__ tt, int B, int S,
                     int H, int NT, float* __restrict__ dpos, float* __restrict__ ws) {
  __shared__ float red[4][64][9];
  const int s = blockIdx.x;
  const int cv = blockIdx.y * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const bool ok = cv * 8 < H;
  float ap[8], at[kPosTypeMaxTypes][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ap[e] = 0.f;
#pragma unroll
    for (int t = 0; t < kPosTypeMaxTypes; ++t) at[t][e] = 0.f;
  }
  if (ok) {
    for (int b = rg; b < B; b += 4) {
      const long r = (long)b * S + s;
      float f[8];
      unpack8(reinterpret_cast<const uint4*>(ds + r * H)[cv], f);
      const int t = tt ? (int)tt[r] : 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) ap[e] += f[e];
#pragma unroll
      for (int q = 0; q < kPosTypeMaxTypes; ++q)
        if (q == t) {
#pragma unroll
          for (int e = 0; e < 8; ++e) at[q][e] += f[e];
        }
    }
  }
  // fixed-order combine of the 4 row groups: positions, then each type
#pragma unroll
  for (int q = -1; q < kPosTypeMaxTypes; ++q) {   // unrolled: at[q] stays in registers
    if (q >= NT) break;
#pragma unroll
    for (int e = 0; e < 8; ++e) red[rg][threadIdx.x & 63][e] = q < 0 ? ap[e] : at[q < 0 ? 0 : q][e];
    __syncthreads();
    if (rg == 0 && ok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = red[0][threadIdx.x][e] + red[1][threadIdx.x][e] + red[2][threadIdx.x][e] +
                        red[3][threadIdx.x][e];
        if (q < 0) dpos[(long)s * H + cv * 8 + e] = v;
        else ws[((long)s * NT + q) * H + cv * 8 + e] = v;
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256)
type_grad_final_kernel(const float* __restrict__ ws, int S, int H, int NT, float* __restrict__ dtyp) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int t = blockIdx.y;
  if (c >= H) return;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += ws[((long)s * NT + t) * H + c];
  dtyp[(long)t * H + c] = v;
}

}  // namespace

int dtf_pos_type_grad_ws_floats(int S, int H, int NT) { return S * NT * H; }

void dtf_pos_type_grad(const bf16_t* ds, const int64_t* tt, int B, int S, int H, int NT,
                       float* dpos, float* dtyp, float* ws, hipStream_t st) {
  if (H % 8) throw std::runtime_error("pos_type_grad: H % 8 != 0");
  if (NT < 1 || NT > kPosTypeMaxTypes) throw std::runtime_error("pos_type_grad: 1..4 token types");
  hipLaunchKernelGGL(pos_type_grad_kernel, dim3(S, (H / 8 + 63) / 64), dim3(256), 0, st, ds, tt,
                     B, S, H, NT, dpos, ws);
  hipLaunchKernelGGL(type_grad_final_kernel, dim3((H + 255) / 256, NT), dim3(256), 0, st, ws, S,
                     H, NT, dtyp);
}

void dtf_segment_sum(const int64_t* sorted_ids, const int64_t* perm, const bf16_t* src,
                     float* out, int T, int H, hipStream_t st) {
  if (H % 4) throw std::runtime_error("segment_sum: H % 4 != 0");
  hipLaunchKernelGGL(segment_sum_kernel, dim3((T * 64 + 255) / 256), dim3(256), 0, st, sorted_ids,
                     perm, src, out, T, H);
}

void dtf_mlm_xent(const bf16_t* logits, const int64_t* labels, const float* weights,
                  const float* denom, int N, int V, int ld, float* loss_rows, bf16_t* grad,
                  hipStream_t st) {
  if ((double)N * ld * 2.0 >= 2147483647.0) throw std::runtime_error("mlm_xent: logits too large");
  if (V < 1 || ld < V) throw std::runtime_error("mlm_xent: row stride below the class count");
  hipLaunchKernelGGL(mlm_xent_kernel, dim3((N * 64 + 255) / 256), dim3(256), 0, st, logits,
                     labels, weights, denom, N, V, ld, loss_rows, grad);
}
