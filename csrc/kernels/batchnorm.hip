// Fused BatchNorm (+residual add) (+ReLU), NHWC bf16 activations, fp32 statistics.
//
// ResNet-50 runs BN after every conv.  The channel axis is innermost (NHWC),
// so one row of M = N*H*W rows holds all C channels contiguously: each lane owns 8 channels
// (one 16-B load) and a block sweeps a contiguous chunk of rows.  Per-channel reductions
// cross workgroups (and therefore XCDs, whose L2s are not coherent), so they are done the
// placement-independent way: per-block partial slabs written with plain stores, combined by a
// SEPARATE finalize launch (the kernel boundary is the release/acquire; cdna_hip_programming.md
// §5 "combine in the NEXT kernel's prologue").  Partial combination is in fp64.
//
// Forward (training):  stats -> finalize(mean, invstd, scale, shift, moving averages) -> apply
// Backward:            reduce(sum dz, sum dz*xhat) -> finalize(dgamma, dbeta, coefs) -> apply
//   with dz = dy * (y > 0) when ReLU was fused, and dx = A*dz + B*x + C per channel.  Without a
//   residual the mask is recomputed from x (fmaf(x, scale, shift) > 0, the forward's exact
//   expression), so the backward never reads y (-2 B/element in both backward passes).
#include <stdexcept>

#include "common.h"

namespace {

constexpr int kThreads = 256;

// rows handled by one block: big enough to amortise the partial slab, small enough to give
// >= ~1024 blocks on ResNet-50's large layers (M = 256*112*112 = 3.2M rows).
// target blocks of a statistics / reduce pass (512 is 1-12 % faster in isolation, -2 % in the
// step: tools/bn_grid_probe.py)
static int g_bn_stats_blocks = 1024;

inline int stats_grid(long M, int C, int* rows_per_block) {
  const int tpr = C / 8;                        // threads per row
  const int rpi = kThreads / tpr;               // rows per block iteration
  long target_blocks = g_bn_stats_blocks;
  long rpb = (M + target_blocks - 1) / target_blocks;
  rpb = ((rpb + rpi - 1) / rpi) * rpi;
  if (rpb < rpi) rpb = rpi;
  *rows_per_block = (int)rpb;
  return (int)((M + rpb - 1) / rpb);
}

// Row-sweep structure shared by the streaming kernels: lane (ro, cg) owns channel group cg
// (8 channels = one 16-B vector) of rows ro, ro + rpi, ... and keeps that group's per-channel
// coefficients in registers for the whole sweep.  Each trip issues the loads of kUnroll rows
// back to back before any use (4-8 independent 16-B loads in flight per lane -- the r1 kernels had
// one, and a 64-bit modulo per vector, and ran at ~4 TB/s).  All offsets are 32-bit vector
// indices (host checks M*C/8 < 2^31).
constexpr int kUnroll = 4;

// ReLU mask source for the backward passes, in order of preference:
//   mask (1 bit per element, written by the forward apply -- the residual BNs, 1/16 of y's bytes)
//   fsc/fsh (recompute fmaf(x, scale, shift) > 0 from x -- BNs without a residual; free)
//   y (the saved output)
DTF_DEV void relu_mask8(float* g, const float* xv, uint32_t mbyte, uint4 yraw, int kind,
                        const float* ksc, const float* ksh) {
  if (kind == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = (mbyte >> i) & 1u ? g[i] : 0.f;
  } else if (kind == 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = __builtin_fmaf(xv[i], ksc[i], ksh[i]) > 0.f ? g[i] : 0.f;
  } else if (kind == 3) {
    float yv[8];
    unpack8(yraw, yv);
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = yv[i] > 0.f ? g[i] : 0.f;
  }
}

DTF_DEV void load8f(const float* __restrict__ p, int cg, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[cg * 2];
  const float4 b = reinterpret_cast<const float4*>(p)[cg * 2 + 1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// MODE 0: forward stats   acc0 += x,           acc1 += x*x
// MODE 1: backward reduce acc0 += dz,          acc1 += dz*(x-mean)*invstd
// MODE 2: MODE 1 for TWO BatchNorms summed before one ReLU (a projection block's residual BN:
//         z = relu(bn(x) + bn_p(xp))): both see the same dz, so one pass reads dz and the mask
//         once and also accumulates acc2 += dz*(xp-mean_p)*invstd_p; the slabs are (acc0, acc1)
//         and (acc0, acc2) -- each exactly what MODE 1 over that BN alone would write
// mkind (MODE 1): 0 no ReLU, 1 bit mask, 2 recompute from x, 3 from y
// 16-B streaming accesses; NT: non-temporal (the tensors are far larger than L2 / MALL and
// every byte is touched once per pass)
typedef uint32_t u32x4_nt __attribute__((ext_vector_type(4)));
template <bool NT>
DTF_DEV uint4 ldv(const uint4* p) {
  if constexpr (NT) {
    const u32x4_nt v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}
template <bool NT>
DTF_DEV void stv(uint4* p, const uint4& v) {
  if constexpr (NT) {
    const u32x4_nt w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4_nt*>(p));
  } else {
    *p = v;
  }
}
static int g_bn_nt = 7;   // bit 0 apply, 1 bwd apply, 2 bwd reduce (tools/bn_bench.py --nt A/B: -6..8 %)

template <int MODE, int MK, bool NT = false>
__global__ void __launch_bounds__(kThreads)
bn_reduce_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                 const bf16_t* __restrict__ y, const uint8_t* __restrict__ mask,
                 const float* __restrict__ mean, const float* __restrict__ invstd, int M, int C,
                 int rows_per_block, int mkind_unused, float* __restrict__ partial,
                 const float* __restrict__ fsc, const float* __restrict__ fsh,
                 const bf16_t* __restrict__ xp, const float* __restrict__ meanp,
                 const float* __restrict__ invstdp, float* __restrict__ partialp) {
  extern __shared__ __attribute__((aligned(16))) float red[];   // [rpi][NQ][C]
  constexpr int NQ = MODE == 2 ? 3 : 2;
  const int tpr = C >> 3;
  const int rpi = kThreads / tpr;
  const int tid = threadIdx.x;
  const int cg = tid % tpr, ro = tid / tpr;
  const bool active = ro < rpi;
  float a0[8], a1[8], a2[8], mu[8], is[8], mup[8], isp[8], ksc[8], ksh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a0[i] = 0.f; a1[i] = 0.f; a2[i] = 0.f; ksc[i] = 0.f; ksh[i] = 0.f; }
  if (MODE >= 1 && active) {
    load8f(mean, cg, mu);
    load8f(invstd, cg, is);
    if (MK == 2) { load8f(fsc, cg, ksc); load8f(fsh, cg, ksh); }
    if (MODE == 2) { load8f(meanp, cg, mup); load8f(invstdp, cg, isp); }
  }
  const int m0 = blockIdx.x * rows_per_block;
  const int m1 = min(m0 + rows_per_block, M);
  const uint4* X4 = reinterpret_cast<const uint4*>(x);
  const uint4* D4 = reinterpret_cast<const uint4*>(dy);
  const uint4* Y4 = reinterpret_cast<const uint4*>(y);
  const uint4* XP4 = reinterpret_cast<const uint4*>(xp);
  if (active) {
    for (int m = m0 + ro; m < m1; m += rpi * kUnroll) {
      uint4 xr[kUnroll], dr[kUnroll], yr[kUnroll], pr[kUnroll];
      uint32_t mb[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int r = m + u * rpi;
        const uint32_t v = (uint32_t)r * tpr + cg;
        const bool ok = r < m1;
        xr[u] = ok ? ldv<NT>(X4 + v) : make_uint4(0, 0, 0, 0);
        if (MODE >= 1) {
          dr[u] = ok ? ldv<NT>(D4 + v) : make_uint4(0, 0, 0, 0);
          mb[u] = (ok && MK == 1) ? (uint32_t)mask[v] : 0u;
          yr[u] = (ok && MK == 3) ? Y4[v] : make_uint4(0, 0, 0, 0);
        }
        if (MODE == 2) pr[u] = ok ? ldv<NT>(XP4 + v) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        float xv[8];
        unpack8(xr[u], xv);        // rows past m1 were loaded as zeros: they add nothing
        if (MODE == 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) { a0[i] += xv[i]; a1[i] += xv[i] * xv[i]; }
        } else {
          float g[8];
          unpack8(dr[u], g);
          relu_mask8(g, xv, mb[u], yr[u], MK, ksc, ksh);
#pragma unroll
          for (int i = 0; i < 8; ++i) { a0[i] += g[i]; a1[i] += g[i] * (xv[i] - mu[i]) * is[i]; }
          if (MODE == 2) {
            float pv[8];
            unpack8(pr[u], pv);
#pragma unroll
            for (int i = 0; i < 8; ++i) a2[i] += g[i] * (pv[i] - mup[i]) * isp[i];
          }
        }
      }
    }
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[(ro * NQ + 0) * C + cg * 8 + i] = a0[i];
      red[(ro * NQ + 1) * C + cg * 8 + i] = a1[i];
      if (MODE == 2) red[(ro * NQ + 2) * C + cg * 8 + i] = a2[i];
    }
  }
  __syncthreads();
  // tree-free final sum: thread t reduces channel-slot t over the rpi row groups
  for (int idx = tid; idx < NQ * C; idx += kThreads) {
    const int which = idx / C, c = idx % C;
    float s = 0.f;
    for (int r = 0; r < rpi; ++r) s += red[(r * NQ + which) * C + c];
    if (which < 2) partial[((long)blockIdx.x * 2 + which) * C + c] = s;
    if (MODE == 2 && which != 1)
      partialp[((long)blockIdx.x * 2 + (which ? 1 : 0)) * C + c] = s;
  }
}

// Two-level fixed-order combine of the G per-block partial slabs (G ~ 1024).  A single
// 32-channel-per-block pass left small-C layers with 2-8 latency-bound blocks (38 us per BN
// call in the r1_v0 profile); stage 1 splits the G rows into S slices over a 2-D grid of
// (C/32) x S blocks, stage 2 (inside the finalize kernels, one thread per channel) adds the S
// fp64 slice sums in order.  Deterministic and placement-independent (kernel boundary = the
// release/acquire between the stages).
inline int combine_slices(int G, int C) {
  // ~1024 combine blocks (the stage-1 layers have G ~ 25k slab rows at b2048: 32 blocks left the
  // GPU idle); stage 2 is block-parallel (8 slices in flight per channel), so S may be large
  const int groups = (C + 31) / 32;
  int S = 1024 / groups;
  if (S > 256) S = 256;
  if (S > G / 8) S = G / 8;
  return S < 1 ? 1 : S;
}

__global__ void __launch_bounds__(256)
bn_combine_kernel(const float* __restrict__ partial, int G, int C, int S,
                  double* __restrict__ level2) {
  __shared__ double red[2][8][32];
  const int cl = threadIdx.x & 31, slot = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  const int j = blockIdx.y;
  const int g0 = (int)((long)j * G / S), g1 = (int)((long)(j + 1) * G / S);
  double s = 0.0, ss = 0.0;
  if (c < C) {
    // loads of 8 rows issued back to back before their (fixed-order) adds
#pragma unroll 8
    for (int g = g0 + slot; g < g1; g += 8) {
      s += partial[((long)g * 2 + 0) * C + c];
      ss += partial[((long)g * 2 + 1) * C + c];
    }
  }
  red[0][slot][cl] = s;
  red[1][slot][cl] = ss;
  __syncthreads();
  if (slot != 0 || c >= C) return;
  s = 0.0;
  ss = 0.0;
  for (int k = 0; k < 8; ++k) { s += red[0][k][cl]; ss += red[1][k][cl]; }
  level2[((long)j * 2 + 0) * C + c] = s;
  level2[((long)j * 2 + 1) * C + c] = ss;
}

// stage 2: block = 32 channels x 8 slice lanes; lane k sums slices k, k + 8, ... in order, the 8
// lane sums are added in order through LDS.  True (with the totals) on the slot-0 threads only.
DTF_DEV bool combine_partials(const double* __restrict__ level2, int S, int C, double* a,
                              double* b, int* c_out) {
  __shared__ double red[2][8][32];
  const int cl = threadIdx.x & 31, slot = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double s = 0.0, ss = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int j = slot; j < S; j += 8) {
      s += level2[((long)j * 2 + 0) * C + c];
      ss += level2[((long)j * 2 + 1) * C + c];
    }
  }
  red[0][slot][cl] = s;
  red[1][slot][cl] = ss;
  __syncthreads();
  if (slot != 0 || c >= C) return false;
  s = 0.0;
  ss = 0.0;
  for (int k = 0; k < 8; ++k) { s += red[0][k][cl]; ss += red[1][k][cl]; }
  *a = s;
  *b = ss;
  *c_out = c;
  return true;
}

__global__ void __launch_bounds__(256)
bn_fwd_finalize_kernel(const double* __restrict__ level2, int S, int C, long M,
                       const float* __restrict__ gamma, const float* __restrict__ beta,
                       float* __restrict__ run_mean, float* __restrict__ run_var, float momentum,
                       float eps, float* __restrict__ mean, float* __restrict__ invstd,
                       float* __restrict__ scale, float* __restrict__ shift) {
  double s, ss;
  int c;
  if (!combine_partials(level2, S, C, &s, &ss, &c)) return;
  const double mu = s / (double)M;
  double var = ss / (double)M - mu * mu;
  if (var < 0) var = 0;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  mean[c] = (float)mu;
  invstd[c] = is;
  const float sc = gamma[c] * is;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mu * sc;
  if (run_mean) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    run_mean[c] = run_mean[c] * momentum + (float)mu * (1.f - momentum);
    run_var[c] = run_var[c] * momentum + (float)unb * (1.f - momentum);
  }
}

__global__ void bn_infer_finalize_kernel(int C, const float* __restrict__ gamma,
                                         const float* __restrict__ beta,
                                         const float* __restrict__ run_mean,
                                         const float* __restrict__ run_var, float eps,
                                         float* __restrict__ mean, float* __restrict__ invstd,
                                         float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = rsqrtf(run_var[c] + eps);
  mean[c] = run_mean[c];
  invstd[c] = is;
  scale[c] = gamma[c] * is;
  shift[c] = beta[c] - run_mean[c] * gamma[c] * is;
}


// y = [relu](x*scale + shift [+ res]); with `mask` also the ReLU bit mask (bit i of byte v =
// element 8v+i > 0) the backward reads instead of y.
// DUAL: res is itself a BatchNorm INPUT (a projection shortcut's conv output) normalised on the
// fly with (rscale, rshift) and rounded to bf16 exactly as its own apply pass would have stored
// it -- the shortcut BN's output is never written or re-read (bit-identical to the two passes).
template <bool NT, bool DUAL = false>
__global__ void __launch_bounds__(kThreads)
bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                bf16_t* __restrict__ y, uint8_t* __restrict__ mask,
                const float* __restrict__ scale, const float* __restrict__ shift, int M, int C,
                int relu, const float* __restrict__ rscale, const float* __restrict__ rshift) {
  const int tpr = C >> 3, rpi = kThreads / tpr;
  const int cg = threadIdx.x % tpr, ro = threadIdx.x / tpr;
  if (ro >= rpi) return;
  float sc[8], sh[8], rsc[8], rsh[8];
  load8f(scale, cg, sc);
  load8f(shift, cg, sh);
  if (DUAL) { load8f(rscale, cg, rsc); load8f(rshift, cg, rsh); }
  const uint4* X4 = reinterpret_cast<const uint4*>(x);
  const uint4* R4 = reinterpret_cast<const uint4*>(res);
  uint4* Y4 = reinterpret_cast<uint4*>(y);
  const int step = gridDim.x * rpi * kUnroll;
  for (int m = blockIdx.x * rpi * kUnroll + ro; m < M; m += step) {
    uint4 xr[kUnroll], rr[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int r = m + u * rpi;
      const uint32_t v = (uint32_t)r * tpr + cg;
      if (r < M) {
        xr[u] = ldv<NT>(X4 + v);
        if (res) rr[u] = ldv<NT>(R4 + v);
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int r = m + u * rpi;
      if (r >= M) break;
      const uint32_t v = (uint32_t)r * tpr + cg;
      float xv[8], o[8];
      unpack8(xr[u], xv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = __builtin_fmaf(xv[i], sc[i], sh[i]);
      if (res) {
        float rv[8];
        unpack8(rr[u], rv);
        if (DUAL) {
#pragma unroll
          for (int i = 0; i < 8; ++i) rv[i] = bf2f(f2bf(__builtin_fmaf(rv[i], rsc[i], rsh[i])));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += rv[i];
      }
      if (relu) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = fmaxf(o[i], 0.f);
      }
      const uint4 packed = pack8(o);
      stv<NT>(Y4 + v, packed);
      if (mask) {
        // the mask is taken from the ROUNDED output, exactly what a y-based mask would see
        float ov[8];
        unpack8(packed, ov);
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) bits |= (ov[i] > 0.f ? 1u : 0u) << i;
        mask[v] = (uint8_t)bits;
      }
    }
  }
}

__global__ void __launch_bounds__(256)
bn_bwd_finalize_kernel(const double* __restrict__ level2, int S, int C, long M,
                       const float* __restrict__ gamma, const float* __restrict__ mean,
                       const float* __restrict__ invstd, float* __restrict__ dgamma,
                       float* __restrict__ dbeta, float* __restrict__ coefA,
                       float* __restrict__ coefB, float* __restrict__ coefC, int accumulate) {
  double sdz, sdzx;
  int c;
  if (!combine_partials(level2, S, C, &sdz, &sdzx, &c)) return;
  const float db = (float)sdz, dg = (float)sdzx;
  if (accumulate) { dgamma[c] += dg; dbeta[c] += db; }
  else { dgamma[c] = dg; dbeta[c] = db; }
  const float is = invstd[c];
  const float k = gamma[c] * is;
  const float invM = 1.f / (float)M;
  const float B = -k * is * dg * invM;
  coefA[c] = k;
  coefB[c] = B;
  coefC[c] = -k * db * invM - B * mean[c];
}

// DUAL: also dxp = Ap*dz + Bp*xp + Cp for the second BatchNorm of a projection block (the one
// whose output was the residual), from the same masked dz (see bn_reduce_kernel MODE 2)
template <int MK, bool NT, bool DUAL = false>
__global__ void __launch_bounds__(kThreads)
bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                    const uint8_t* __restrict__ mask, const bf16_t* __restrict__ x,
                    const float* __restrict__ cA, const float* __restrict__ cB,
                    const float* __restrict__ cC, bf16_t* __restrict__ dx,
                    bf16_t* __restrict__ dres, int M, int C, int mkind_unused,
                    const float* __restrict__ fsc, const float* __restrict__ fsh,
                    const bf16_t* __restrict__ xp, const float* __restrict__ cAp,
                    const float* __restrict__ cBp, const float* __restrict__ cCp,
                    bf16_t* __restrict__ dxp) {
  const int tpr = C >> 3, rpi = kThreads / tpr;
  const int cg = threadIdx.x % tpr, ro = threadIdx.x / tpr;
  if (ro >= rpi) return;
  float ka[8], kb[8], kc[8], ksc[8], ksh[8], pa[8], pb[8], pc[8];
  load8f(cA, cg, ka);
  load8f(cB, cg, kb);
  load8f(cC, cg, kc);
  if (MK == 2) { load8f(fsc, cg, ksc); load8f(fsh, cg, ksh); }
  if (DUAL) { load8f(cAp, cg, pa); load8f(cBp, cg, pb); load8f(cCp, cg, pc); }
  const uint4* XP4 = reinterpret_cast<const uint4*>(xp);
  uint4* DXP4 = reinterpret_cast<uint4*>(dxp);
  const uint4* D4 = reinterpret_cast<const uint4*>(dy);
  const uint4* X4 = reinterpret_cast<const uint4*>(x);
  const uint4* Y4 = reinterpret_cast<const uint4*>(y);
  uint4* DX4 = reinterpret_cast<uint4*>(dx);
  uint4* DR4 = reinterpret_cast<uint4*>(dres);
  const int step = gridDim.x * rpi * kUnroll;
  // DUAL without dx: a fused conv backward forms d(x) itself (ops/native.py _LazyBnDx); only the
  // shortcut's dxp is written and x is not read
  const bool want_dx = !DUAL || dx != nullptr;
  for (int m = blockIdx.x * rpi * kUnroll + ro; m < M; m += step) {
    uint4 dr[kUnroll], xr[kUnroll], yr[kUnroll], pr[kUnroll];
    uint32_t mb[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int r = m + u * rpi;
      const uint32_t v = (uint32_t)r * tpr + cg;
      if (r < M) {
        dr[u] = ldv<NT>(D4 + v);
        xr[u] = want_dx ? ldv<NT>(X4 + v) : make_uint4(0, 0, 0, 0);
        if (MK == 1) mb[u] = mask[v];
        if (MK == 3) yr[u] = Y4[v];
        if (DUAL) pr[u] = ldv<NT>(XP4 + v);
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int r = m + u * rpi;
      if (r >= M) break;
      const uint32_t v = (uint32_t)r * tpr + cg;
      float g[8], xv[8], o[8];
      unpack8(dr[u], g);
      unpack8(xr[u], xv);
      relu_mask8(g, xv, MK == 1 ? mb[u] : 0u, MK == 3 ? yr[u] : make_uint4(0, 0, 0, 0),
                 MK, ksc, ksh);
      if (dres) stv<NT>(DR4 + v, pack8(g));
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = bn_bwd_dx(ka[i], g[i], kb[i], xv[i], kc[i]);
      if (want_dx) stv<NT>(DX4 + v, pack8(o));
      if (DUAL) {
        float pv[8];
        unpack8(pr[u], pv);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = bn_bwd_dx(pa[i], g[i], pb[i], pv[i], pc[i]);
        stv<NT>(DXP4 + v, pack8(o));
      }
    }
  }
}

inline int mask_kind(int relu, const uint8_t* mask, const float* fsc, const float* fsh,
                     const bf16_t* y) {
  if (!relu) return 0;
  if (mask) return 1;
  if (fsc && fsh) return 2;
  if (y) return 3;
  throw std::runtime_error("bn_bwd: relu mask needs a bit mask, y or scale/shift");
}

inline void check_rows(long M, int C) {
  if (C % 8 || C > 2048 || M * (long)(C / 8) >= 2147483647L)
    throw std::runtime_error("batch_norm: unsupported shape (C % 8, C <= 2048, M*C/8 < 2^31)");
}

// override of the row-sweep grid caps below (0 = per-kernel defaults; tools/bn_grid_probe.py)
static int g_bn_grid_cap = 0;

// blocks for a row sweep (grid-stride): up to 8 per CU, at most `cap`.  Isolated sweeps of the
// ResNet-50 b1984 shapes run 2-12 % faster at 1-2 blocks per CU (tools/bn_grid_probe.py), but
// inside the training step the same caps moved the BN kernels by -4..+5 % and the step not at
// all (profiles/measurements/r3_bn_grid_probe_b1984.jsonl), so the caps stay at 8 per CU.
constexpr int kSweepApply = 2048, kSweepApplyRes = 2048, kSweepBwd = 2048;
inline int sweep_grid(long M, int C, int cap) {
  const int rpi = kThreads / (C / 8);
  long g = (M + (long)rpi * kUnroll - 1) / ((long)rpi * kUnroll);
  if (g_bn_grid_cap > 0) cap = g_bn_grid_cap;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

// out = dy * relu_mask (1 bit per element): materialises a lazily kept residual gradient on the
// rare paths whose consumer cannot form it in an epilogue (see ops/native.py _MaskedGrad)
__global__ void __launch_bounds__(kThreads)
relu_mask_apply_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ mask,
                       bf16_t* __restrict__ out, long nv) {
  const uint4* D4 = reinterpret_cast<const uint4*>(dy);
  uint4* O4 = reinterpret_cast<uint4*>(out);
  for (long v = (long)blockIdx.x * kThreads + threadIdx.x; v < nv; v += (long)gridDim.x * kThreads) {
    float g[8];
    unpack8(D4[v], g);
    relu_mask8(g, nullptr, mask[v], make_uint4(0, 0, 0, 0), 1, nullptr, nullptr);
    O4[v] = pack8(g);
  }
}

}  // namespace

void dtf_relu_mask_apply(const bf16_t* dy, const uint8_t* mask, bf16_t* out, long n,
                         hipStream_t st) {
  if (n % 8) throw std::runtime_error("relu_mask_apply: n must be a multiple of 8");
  const long nv = n / 8;
  long g = (nv + kThreads - 1) / kThreads;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(relu_mask_apply_kernel, dim3((int)g), dim3(kThreads), 0, st, dy, mask, out,
                     nv);
}

// ------------------------------------------------------------------ launchers (host)
int dtf_bn_partial_blocks(long M, int C) {
  int rpb;
  return stats_grid(M, C, &rpb);
}

void dtf_bn_fwd_stats(const bf16_t* x, long M, int C, float* partial, hipStream_t st) {
  check_rows(M, C);
  int rpb;
  const int G = stats_grid(M, C, &rpb);
  const int rpi = kThreads / (C / 8);
  const size_t lds = (size_t)rpi * 2 * C * sizeof(float);
  hipLaunchKernelGGL((bn_reduce_kernel<0, 0>), dim3(G), dim3(kThreads), lds, st, x, nullptr, nullptr,
                     nullptr, nullptr, nullptr, (int)M, C, rpb, 0, partial, nullptr, nullptr,
                     nullptr, nullptr, nullptr, nullptr);
}

void dtf_bn_fwd_finalize_g(const float* partial, int G, long M, int C, const float* gamma,
                           const float* beta, float* run_mean, float* run_var, float momentum,
                           float eps, float* mean, float* invstd, float* scale, float* shift,
                           hipStream_t st) {
  const int S = combine_slices(G, C);
  double* level2 = reinterpret_cast<double*>(const_cast<float*>(partial) + (long)G * 2 * C);
  hipLaunchKernelGGL(bn_combine_kernel, dim3((C + 31) / 32, S), dim3(256), 0, st, partial, G, C,
                     S, level2);
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 31) / 32), dim3(256), 0, st, level2, S,
                     C, M, gamma, beta, run_mean, run_var, momentum, eps, mean, invstd, scale,
                     shift);
}

void dtf_bn_fwd_finalize(const float* partial, long M, int C, const float* gamma,
                         const float* beta, float* run_mean, float* run_var, float momentum,
                         float eps, float* mean, float* invstd, float* scale, float* shift,
                         hipStream_t st) {
  int rpb;
  const int G = stats_grid(M, C, &rpb);
  dtf_bn_fwd_finalize_g(partial, G, M, C, gamma, beta, run_mean, run_var, momentum, eps, mean,
                        invstd, scale, shift, st);
}

// floats of workspace for G partial slabs + the fp64 combine slices
long dtf_bn_workspace_floats_g(int G, int C) {
  return (long)G * 2 * C + 2L * combine_slices(G, C) * 2 * C;
}

// floats of workspace a stats/reduce + finalize pair needs: G partial slabs + S fp64 slices
long dtf_bn_workspace_floats(long M, int C) {
  int rpb;
  return dtf_bn_workspace_floats_g(stats_grid(M, C, &rpb), C);
}

void dtf_bn_infer_finalize(int C, const float* gamma, const float* beta, const float* run_mean,
                           const float* run_var, float eps, float* mean, float* invstd,
                           float* scale, float* shift, hipStream_t st) {
  hipLaunchKernelGGL(bn_infer_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma,
                     beta, run_mean, run_var, eps, mean, invstd, scale, shift);
}

void dtf_bn_apply(const bf16_t* x, const bf16_t* res, bf16_t* y, uint8_t* mask,
                  const float* scale, const float* shift, long M, int C, int relu,
                  hipStream_t st) {
  check_rows(M, C);
  const int cap = res ? kSweepApplyRes : kSweepApply;
  if (g_bn_nt & 1)
    hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(sweep_grid(M, C, cap)), dim3(kThreads), 0, st, x,
                       res, y, mask, scale, shift, (int)M, C, relu, nullptr, nullptr);
  else
    hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(sweep_grid(M, C, cap)), dim3(kThreads), 0, st, x,
                       res, y, mask, scale, shift, (int)M, C, relu, nullptr, nullptr);
}

// y = relu(bn(x) + bn_p(xp)) (+ ReLU bit mask): a projection block's two BatchNorms in one pass
void dtf_bn_apply_dual(const bf16_t* x, const bf16_t* xp, bf16_t* y, uint8_t* mask,
                       const float* scale, const float* shift, const float* pscale,
                       const float* pshift, long M, int C, int relu, hipStream_t st) {
  check_rows(M, C);
  if (!xp || !pscale || !pshift) throw std::runtime_error("bn_apply_dual: missing operands");
  if (g_bn_nt & 1)
    hipLaunchKernelGGL((bn_apply_kernel<true, true>), dim3(sweep_grid(M, C, kSweepApplyRes)), dim3(kThreads), 0, st,
                       x, xp, y, mask, scale, shift, (int)M, C, relu, pscale, pshift);
  else
    hipLaunchKernelGGL((bn_apply_kernel<false, true>), dim3(sweep_grid(M, C, kSweepApplyRes)), dim3(kThreads), 0,
                       st, x, xp, y, mask, scale, shift, (int)M, C, relu, pscale, pshift);
}

void dtf_bn_set_nt(int v) { g_bn_nt = v; }
void dtf_bn_set_grid_cap(int v) { g_bn_grid_cap = v; }
void dtf_bn_set_stats_blocks(int v) { g_bn_stats_blocks = v > 0 ? v : 1024; }

void dtf_bn_bwd_reduce(const bf16_t* dy, const bf16_t* y, const uint8_t* mask, const bf16_t* x,
                       const float* mean, const float* invstd, long M, int C, int relu,
                       float* partial, const float* fsc, const float* fsh, hipStream_t st) {
  check_rows(M, C);
  const int mk = mask_kind(relu, mask, fsc, fsh, y);
  int rpb;
  const int G = stats_grid(M, C, &rpb);
  const int rpi = kThreads / (C / 8);
  const size_t lds = (size_t)rpi * 2 * C * sizeof(float);
  // mask kind is a template parameter: the unused mask operands take no registers
#define DTF_BN_RED(MK_)                                                                    \
  if (g_bn_nt & 4)                                                                         \
    hipLaunchKernelGGL((bn_reduce_kernel<1, MK_, true>), dim3(G), dim3(kThreads), lds, st, x, dy, \
                       y, mask, mean, invstd, (int)M, C, rpb, mk, partial, fsc, fsh, nullptr,   \
                       nullptr, nullptr, nullptr);                                          \
  else                                                                                     \
    hipLaunchKernelGGL((bn_reduce_kernel<1, MK_>), dim3(G), dim3(kThreads), lds, st, x, dy, y,   \
                       mask, mean, invstd, (int)M, C, rpb, mk, partial, fsc, fsh, nullptr,      \
                       nullptr, nullptr, nullptr)
  switch (mk) {
    case 0: DTF_BN_RED(0); break;
    case 1: DTF_BN_RED(1); break;
    case 2: DTF_BN_RED(2); break;
    default: DTF_BN_RED(3); break;
  }
#undef DTF_BN_RED
}

void dtf_bn_bwd_finalize_g(const float* partial, int G, long M, int C, const float* gamma,
                           const float* mean, const float* invstd, float* dgamma, float* dbeta,
                           float* coefA, float* coefB, float* coefC, int accumulate,
                           hipStream_t st) {
  const int S = combine_slices(G, C);
  double* level2 = reinterpret_cast<double*>(const_cast<float*>(partial) + (long)G * 2 * C);
  hipLaunchKernelGGL(bn_combine_kernel, dim3((C + 31) / 32, S), dim3(256), 0, st, partial, G, C,
                     S, level2);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 31) / 32), dim3(256), 0, st, level2, S,
                     C, M, gamma, mean, invstd, dgamma, dbeta, coefA, coefB, coefC, accumulate);
}

void dtf_bn_bwd_finalize(const float* partial, long M, int C, const float* gamma,
                         const float* mean, const float* invstd, float* dgamma, float* dbeta,
                         float* coefA, float* coefB, float* coefC, int accumulate,
                         hipStream_t st) {
  int rpb;
  const int G = stats_grid(M, C, &rpb);
  const int S = combine_slices(G, C);
  double* level2 = reinterpret_cast<double*>(const_cast<float*>(partial) + (long)G * 2 * C);
  hipLaunchKernelGGL(bn_combine_kernel, dim3((C + 31) / 32, S), dim3(256), 0, st, partial, G, C,
                     S, level2);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 31) / 32), dim3(256), 0, st, level2, S,
                     C, M, gamma, mean, invstd, dgamma, dbeta, coefA, coefB, coefC, accumulate);
}

void dtf_bn_bwd_apply(const bf16_t* dy, const bf16_t* y, const uint8_t* mask, const bf16_t* x,
                      const float* cA, const float* cB, const float* cC, bf16_t* dx,
                      bf16_t* dres, long M, int C, int relu, const float* fsc, const float* fsh,
                      hipStream_t st) {
  check_rows(M, C);
  const int mk = mask_kind(relu, mask, fsc, fsh, y);
#define DTF_BN_BWD(MK_)                                                                    \
  if (g_bn_nt & 2)                                                                         \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<MK_, true>), dim3(sweep_grid(M, C, kSweepBwd)), dim3(kThreads), \
                       0, st, dy, y, mask, x, cA, cB, cC, dx, dres, (int)M, C, mk, fsc, fsh,   \
                       nullptr, nullptr, nullptr, nullptr, nullptr);                        \
  else                                                                                     \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<MK_, false>), dim3(sweep_grid(M, C, kSweepBwd)), dim3(kThreads), \
                       0, st, dy, y, mask, x, cA, cB, cC, dx, dres, (int)M, C, mk, fsc, fsh,   \
                       nullptr, nullptr, nullptr, nullptr, nullptr)
  switch (mk) {
    case 0: DTF_BN_BWD(0); break;
    case 1: DTF_BN_BWD(1); break;
    case 2: DTF_BN_BWD(2); break;
    default: DTF_BN_BWD(3); break;
  }
#undef DTF_BN_BWD
}

// Backward of y = relu(bn(x) + bn_p(xp)) with the forward's ReLU bit mask: one reduce pass for
// both BatchNorms' sums (dz and the mask read once), then -- after the two finalizes -- one apply
// pass writing dx and dxp.  Each slab / output is bit-identical to the single-BN passes.
void dtf_bn_bwd_reduce_dual(const bf16_t* dy, const uint8_t* mask, const bf16_t* x,
                            const float* mean, const float* invstd, const bf16_t* xp,
                            const float* meanp, const float* invstdp, long M, int C,
                            float* partial, float* partialp, hipStream_t st) {
  check_rows(M, C);
  if (!mask) throw std::runtime_error("bn_bwd_reduce_dual: needs the forward ReLU bit mask");
  int rpb;
  const int G = stats_grid(M, C, &rpb);
  const int rpi = kThreads / (C / 8);
  const size_t lds = (size_t)rpi * 3 * C * sizeof(float);
  if (g_bn_nt & 4)
    hipLaunchKernelGGL((bn_reduce_kernel<2, 1, true>), dim3(G), dim3(kThreads), lds, st, x, dy,
                       nullptr, mask, mean, invstd, (int)M, C, rpb, 1, partial, nullptr, nullptr,
                       xp, meanp, invstdp, partialp);
  else
    hipLaunchKernelGGL((bn_reduce_kernel<2, 1>), dim3(G), dim3(kThreads), lds, st, x, dy, nullptr,
                       mask, mean, invstd, (int)M, C, rpb, 1, partial, nullptr, nullptr, xp, meanp,
                       invstdp, partialp);
}

void dtf_bn_bwd_apply_dual(const bf16_t* dy, const uint8_t* mask, const bf16_t* x,
                           const float* cA, const float* cB, const float* cC, bf16_t* dx,
                           const bf16_t* xp, const float* cAp, const float* cBp,
                           const float* cCp, bf16_t* dxp, long M, int C, hipStream_t st) {
  check_rows(M, C);
  if (!mask) throw std::runtime_error("bn_bwd_apply_dual: needs the forward ReLU bit mask");
  if (g_bn_nt & 2)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<1, true, true>), dim3(sweep_grid(M, C, kSweepBwd)), dim3(kThreads),
                       0, st, dy, nullptr, mask, x, cA, cB, cC, dx, nullptr, (int)M, C, 1, nullptr,
                       nullptr, xp, cAp, cBp, cCp, dxp);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<1, false, true>), dim3(sweep_grid(M, C, kSweepBwd)),
                       dim3(kThreads), 0, st, dy, nullptr, mask, x, cA, cB, cC, dx, nullptr, (int)M,
                       C, 1, nullptr, nullptr, xp, cAp, cBp, cCp, dxp);
}
