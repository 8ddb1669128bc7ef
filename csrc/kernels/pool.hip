// Max-pool (any k/stride/pad, NHWC) forward with stored window-argmax, gather-form backward
// (no atomics: each input pixel sums the <= ceil(k/s)^2 outputs whose argmax selected it),
// and global average pool forward/backward.  SURVEY.md K4/K4b/K6 (MNIST 2x2/2) and N-K3
// (ResNet-50 3x3/2 pad 1, 7x7 global average).  8 channels (16 B) per lane.
#include "common.h"

#include <stdexcept>

namespace {
constexpr int kT = 256;

// IT: index type of the flat element loop -- 32-bit whenever the tensor allows (a 64-bit
// divide/modulo is a ~100-instruction software sequence per element on CDNA)
template <typename IT>
__global__ void __launch_bounds__(kT)
maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                   uint8_t* __restrict__ arg, int N, int H, int W, int C, int P, int Q, int kh,
                   int kw, int sh, int sw, int ph, int pw) {
  const IT cv = (IT)(C >> 3);
  const IT total = (IT)N * P * Q * cv;
  for (IT i = (IT)blockIdx.x * kT + threadIdx.x; i < total; i += (IT)gridDim.x * kT) {
    const int cg = (int)(i % cv);
    IT t = i / cv;
    const int q = (int)(t % (IT)Q); t /= (IT)Q;
    const int p = (int)(t % (IT)P);
    const int n = (int)(t / (IT)P);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int r = 0; r < kh; ++r) {
      const int h = p * sh - ph + r;
      if (h < 0 || h >= H) continue;
      for (int s = 0; s < kw; ++s) {
        const int w = q * sw - pw + s;
        if (w < 0 || w >= W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((long)n * H + h) * W + w) * C + cg * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > best[j]) { best[j] = v[j]; bi[j] = (uint8_t)(r * kw + s); }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    reinterpret_cast<uint2*>(arg)[i] = a;
  }
}

// BatchNorm apply + ReLU + max-pool in one pass (the ResNet stem): the window maximum of
// bf16(relu(x * scale + shift)) -- exactly the values bn_apply would have written, rounded the
// same way -- so the 112x112x64 BN output is never stored or re-read.  The BN backward
// recomputes its ReLU mask from x, and the pool backward needs only `arg`.
template <typename IT>
__global__ void __launch_bounds__(kT)
bn_relu_maxpool_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                           const float* __restrict__ shift, bf16_t* __restrict__ y,
                           uint8_t* __restrict__ arg, int N, int H, int W, int C, int P, int Q,
                           int kh, int kw, int sh, int sw, int ph, int pw) {
  const IT cv = (IT)(C >> 3);
  const IT total = (IT)N * P * Q * cv;
  for (IT i = (IT)blockIdx.x * kT + threadIdx.x; i < total; i += (IT)gridDim.x * kT) {
    const int cg = (int)(i % cv);
    IT t = i / cv;
    const int q = (int)(t % (IT)Q); t /= (IT)Q;
    const int p = (int)(t % (IT)P);
    const int n = (int)(t / (IT)P);
    float sc[8], sf[8], best[8];
    uint8_t bi[8];
    const float4* S4 = reinterpret_cast<const float4*>(scale + cg * 8);
    const float4* F4 = reinterpret_cast<const float4*>(shift + cg * 8);
    const float4 s0 = S4[0], s1 = S4[1], f0 = F4[0], f1 = F4[1];
    sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
    sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    sf[0] = f0.x; sf[1] = f0.y; sf[2] = f0.z; sf[3] = f0.w;
    sf[4] = f1.x; sf[5] = f1.y; sf[6] = f1.z; sf[7] = f1.w;
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int r = 0; r < kh; ++r) {
      const int h = p * sh - ph + r;
      if (h < 0 || h >= H) continue;
      for (int s = 0; s < kw; ++s) {
        const int w = q * sw - pw + s;
        if (w < 0 || w >= W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((long)n * H + h) * W + w) * C + cg * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = bf2f(f2bf(fmaxf(__builtin_fmaf(v[j], sc[j], sf[j]), 0.f)));
          if (o > best[j]) { best[j] = o; bi[j] = (uint8_t)(r * kw + s); }
        }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    reinterpret_cast<uint2*>(arg)[i] = a;
  }
}

// The 3x3 / stride-2 / pad-1 case of the kernel above (the ResNet stem): the window is unrolled
// so its nine 16-B loads are all in flight before the first max (the generic loop waits on each
// in turn), and the channel group -- fixed per lane since kT % (C / 8) == 0 -- loads its scale /
// shift once.  Same visiting order and tie rule: bit-identical outputs and argmax bytes.
__global__ void __launch_bounds__(kT)
bn_relu_maxpool3s2_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                              const float* __restrict__ shift, bf16_t* __restrict__ y,
                              uint8_t* __restrict__ arg, int N, int H, int W, int C, int P, int Q) {
  const uint32_t cv = (uint32_t)(C >> 3);
  const uint32_t total = (uint32_t)N * P * Q * cv;
  const int cg = (int)((blockIdx.x * kT + threadIdx.x) % cv);
  float sc[8], sf[8];
  {
    const float4* S4 = reinterpret_cast<const float4*>(scale + cg * 8);
    const float4* F4 = reinterpret_cast<const float4*>(shift + cg * 8);
    const float4 s0 = S4[0], s1 = S4[1], f0 = F4[0], f1 = F4[1];
    sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
    sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    sf[0] = f0.x; sf[1] = f0.y; sf[2] = f0.z; sf[3] = f0.w;
    sf[4] = f1.x; sf[5] = f1.y; sf[6] = f1.z; sf[7] = f1.w;
  }
  const uint4* X4 = reinterpret_cast<const uint4*>(x);
  for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < total; i += gridDim.x * kT) {
    uint32_t t = i / cv;
    const int q = (int)(t % (uint32_t)Q); t /= (uint32_t)Q;
    const int p = (int)(t % (uint32_t)P);
    const int n = (int)(t / (uint32_t)P);
    const int h0 = 2 * p - 1, w0 = 2 * q - 1;
    uint4 v[9];
    bool ok[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int h = h0 + r, w = w0 + s;
        ok[r * 3 + s] = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        const int hc = ok[r * 3 + s] ? h : 0, wc = ok[r * 3 + s] ? w : 0;
        v[r * 3 + s] = X4[(((uint32_t)n * H + hc) * W + wc) * cv + cg];
      }
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (!ok[k]) continue;
      float f[8];
      unpack8(v[k], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float o = bf2f(f2bf(fmaxf(__builtin_fmaf(f[j], sc[j], sf[j]), 0.f)));
        if (o > best[j]) { best[j] = o; bi[j] = (uint32_t)k; }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    uint2 a;
    a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    reinterpret_cast<uint2*>(arg)[i] = a;
  }
}

template <typename IT>
__global__ void __launch_bounds__(kT)
maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                   bf16_t* __restrict__ dx, int N, int H, int W, int C, int P, int Q, int kh,
                   int kw, int sh, int sw, int ph, int pw) {
  const IT cv = (IT)(C >> 3);
  const IT total = (IT)N * H * W * cv;
  for (IT i = (IT)blockIdx.x * kT + threadIdx.x; i < total; i += (IT)gridDim.x * kT) {
    const int cg = (int)(i % cv);
    IT t = i / cv;
    const int w = (int)(t % (IT)W); t /= (IT)W;
    const int h = (int)(t % (IT)H);
    const int n = (int)(t / (IT)H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // outputs p with p*sh - ph <= h <= p*sh - ph + kh - 1
    int p0 = h + ph - kh + 1;
    p0 = p0 <= 0 ? 0 : (p0 + sh - 1) / sh;
    int p1 = (h + ph) / sh;
    if (p1 > P - 1) p1 = P - 1;
    int q0 = w + pw - kw + 1;
    q0 = q0 <= 0 ? 0 : (q0 + sw - 1) / sw;
    int q1 = (w + pw) / sw;
    if (q1 > Q - 1) q1 = Q - 1;
    for (int p = p0; p <= p1; ++p) {
      const int r = h - (p * sh - ph);
      for (int q = q0; q <= q1; ++q) {
        const int s = w - (q * sw - pw);
        const uint8_t me = (uint8_t)(r * kw + s);
        const long o = (((long)n * P + p) * Q + q) * cv + cg;
        float g[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[o], g);
        const uint2 a = reinterpret_cast<const uint2*>(arg)[o];
        const uint32_t aw[2] = {a.x, a.y};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((aw[j >> 2] >> ((j & 3) * 8)) & 0xff) == me) acc[j] += g[j];
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(acc);
  }
}

// global average pool: one lane = 8 channels of one image, loops over H*W rows.
__global__ void __launch_bounds__(kT)
gap_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N, int HW, int C) {
  const int cv = C >> 3;
  const long total = (long)N * cv;
  const long i = (long)blockIdx.x * kT + threadIdx.x;
  if (i >= total) return;
  const int cg = (int)(i % cv);
  const int n = (int)(i / cv);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const bf16_t* base = x + (long)n * HW * C + cg * 8;
  for (int r = 0; r < HW; ++r) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(base + (long)r * C), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  reinterpret_cast<uint4*>(y)[i] = pack8(acc);
}

__global__ void __launch_bounds__(kT)
gap_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int N, int HW, int C) {
  const int cv = C >> 3;
  const long total = (long)N * HW * cv;
  const float inv = 1.f / (float)HW;
  for (long i = (long)blockIdx.x * kT + threadIdx.x; i < total; i += (long)gridDim.x * kT) {
    const int cg = (int)(i % cv);
    const int n = (int)(i / ((long)HW * cv));
    float g[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[(long)n * cv + cg], g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= inv;
    reinterpret_cast<uint4*>(dx)[i] = pack8(g);
  }
}

// 3x3 / stride 2 / pad 1 backward (the ResNet stem pool), blocked: one lane owns a 2x2 block
// of input pixels x 8 channels, which together read exactly output rows {a, a+1} x cols
// {b, b+1}; each output (dy, argmax) is loaded once instead of once per input pixel it covers
// (2.25x on average).  Same accumulation order as maxpool_bwd_kernel (p, then q ascending).
__global__ void __launch_bounds__(kT)
maxpool3s2_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                      bf16_t* __restrict__ dx, int N, int H, int W, int C, int P, int Q) {
  const int cv = C >> 3;
  const int HB = (H + 1) >> 1, WB = (W + 1) >> 1;
  const uint32_t total = (uint32_t)N * HB * WB * cv;
  for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < total; i += gridDim.x * kT) {
    const int cg = (int)(i % cv);
    uint32_t t = i / cv;
    const int b = (int)(t % WB); t /= WB;
    const int a = (int)(t % HB);
    const int n = (int)(t / HB);
    float acc[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
#pragma unroll
    for (int da = 0; da < 2; ++da) {
      const int p = a + da;
      if (p >= P) continue;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const int q = b + db;
        if (q >= Q) continue;
        const long o = (((long)n * P + p) * Q + q) * cv + cg;
        float g[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[o], g);
        const uint2 am = reinterpret_cast<const uint2*>(arg)[o];
        const uint32_t aw[2] = {am.x, am.y};
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int r = ii - 2 * da + 1, s = jj - 2 * db + 1;
            if (r < 0 || r > 2 || s < 0 || s > 2) continue;     // compile-time after unrolling
            const uint32_t me = (uint32_t)(r * 3 + s);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (((aw[e >> 2] >> ((e & 3) * 8)) & 0xffu) == me) acc[ii * 2 + jj][e] += g[e];
          }
      }
    }
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int h = 2 * a + ii;
      if (h >= H) continue;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int w = 2 * b + jj;
        if (w >= W) continue;
        reinterpret_cast<uint4*>(dx)[(((long)n * H + h) * W + w) * cv + cg] = pack8(acc[ii * 2 + jj]);
      }
    }
  }
}

// Stem backward without the pooled gradient's full-size round trip: the 3x3/2 pool gather of
// maxpool3s2_bwd_kernel (same 2x2 input blocks, same fp32 order, same bf16 rounding) feeds the
// BatchNorm backward directly -- the reduce pass (per-channel sum(dz), sum(dz * xhat) into one
// [2][C] row per block, combined by bn_bwd_finalize_g) and the apply pass (dx = A dz + B x + C)
// each regather it instead of reading a materialised 112x112x64 d(BN output).  The ReLU mask is
// recomputed from x with the forward scale / shift.  Requires 256 % (C / 8) == 0 so every lane
// keeps one channel group across its grid-stride loop.
// g[ii * 2 + jj] = the pooled gradient of input pixel (2a + ii, 2b + jj): the sum over the up to
// four output windows (a + da, b + db) whose argmax byte names that pixel.  dyr / amr hold the
// windows' (clamped, preloaded) gradients and argmax words; windows past P / Q are skipped.
// pool3s2_gather (common.h): the 2 x 2 conv pixels' gradient gathered from the 4 pooled outputs

DTF_DEV void load8(const float* __restrict__ p, int cg, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p + cg * 8)[0];
  const float4 b = reinterpret_cast<const float4*>(p + cg * 8)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <bool APPLY>
__global__ void __launch_bounds__(kT)
pool3s2_bn_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                      const bf16_t* __restrict__ x, const float* __restrict__ c0,
                      const float* __restrict__ c1, const float* __restrict__ c2,
                      const float* __restrict__ fsc, const float* __restrict__ fsh,
                      bf16_t* __restrict__ dx, float* __restrict__ partial, int N, int H, int W,
                      int C, int P, int Q) {
  // REDUCE: c0 = mean, c1 = invstd;  APPLY: c0/c1/c2 = A/B/C coefficients
  const int cv = C >> 3;
  const int HB = (H + 1) >> 1, WB = (W + 1) >> 1;
  const uint32_t total = (uint32_t)N * HB * WB * cv;
  const int cg = (int)((blockIdx.x * kT + threadIdx.x) % cv);   // fixed: kT % cv == 0
  float k0[8], k1[8], k2[8], ksc[8], ksh[8], a0[8], a1[8];
  load8(c0, cg, k0);
  load8(c1, cg, k1);
  if (APPLY) load8(c2, cg, k2);
  load8(fsc, cg, ksc);
  load8(fsh, cg, ksh);
#pragma unroll
  for (int e = 0; e < 8; ++e) { a0[e] = 0.f; a1[e] = 0.f; }
  for (uint32_t i = blockIdx.x * kT + threadIdx.x; i < total; i += gridDim.x * kT) {
    uint32_t t = i / cv;
    const int b = (int)(t % WB); t /= WB;
    const int a = (int)(t % HB);
    const int n = (int)(t / HB);
    // every load of the 2x2 block up front (clamped addresses): 12 requests in flight per lane
    // instead of a chain of dependent ones behind the boundary branches
    uint4 dyr[4], xr[4];
    uint2 amr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = min(a + (k >> 1), P - 1), q = min(b + (k & 1), Q - 1);
      const uint32_t o = (((uint32_t)n * P + p) * Q + q) * cv + cg;
      dyr[k] = reinterpret_cast<const uint4*>(dy)[o];
      amr[k] = reinterpret_cast<const uint2*>(arg)[o];
      const int h = min(2 * a + (k >> 1), H - 1), w = min(2 * b + (k & 1), W - 1);
      xr[k] = reinterpret_cast<const uint4*>(x)[(((uint32_t)n * H + h) * W + w) * cv + cg];
    }
    float g[4][8];
    pool3s2_gather(dyr, amr, a, b, P, Q, g);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int h = 2 * a + ii;
      if (h >= H) continue;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int w = 2 * b + jj;
        if (w >= W) continue;
        const uint32_t v = (((uint32_t)n * H + h) * W + w) * cv + cg;
        float xv[8];
        unpack8(xr[ii * 2 + jj], xv);
        float* gk = g[ii * 2 + jj];
#pragma unroll
        for (int e = 0; e < 8; ++e) gk[e] = __builtin_fmaf(xv[e], ksc[e], ksh[e]) > 0.f ? gk[e] : 0.f;
        if (APPLY) {
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = bn_bwd_dx(k0[e], gk[e], k1[e], xv[e], k2[e]);
          reinterpret_cast<uint4*>(dx)[v] = pack8(o);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) { a0[e] += gk[e]; a1[e] += gk[e] * (xv[e] - k0[e]) * k1[e]; }
        }
      }
    }
  }
  if (!APPLY) {
    __shared__ float red[kT][17];
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[threadIdx.x][e] = a0[e]; red[threadIdx.x][8 + e] = a1[e]; }
    __syncthreads();
    // channel c = cg*8 + e, quantity q: fixed-order sum over the lanes of channel group cg
    for (int idx = threadIdx.x; idx < 2 * C; idx += kT) {
      const int q = idx / C, c = idx % C, g8 = c >> 3, e = c & 7;
      float sacc = 0.f;
      for (int l = g8; l < kT; l += cv) sacc += red[l][q * 8 + e];
      partial[((long)blockIdx.x * 2 + q) * C + c] = sacc;
    }
  }
}

inline int grid_for(long n) {
  long g = (n + kT - 1) / kT;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}
// Space-to-depth input of the strided stem (ops/reference.py space_to_depth_operands), one pass:
// xs[n, i, j, (a*s + b)*cp + ch] = x[n, s*i + a - pad, s*j + b - pad, ch] (zero outside the image
// and for ch >= C).  One lane per output pixel; cp*s*s = 16 channels = 32 B per lane.  Replaces
// torch's zero-fill + padded copy + permute copy (three full passes over the padded image).
template <int SS, int CP>
__global__ void __launch_bounds__(kT)
s2d_input_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xs, int N, int H, int W,
                 int C, int Ho, int Wo, int pad) {
  constexpr int OC = SS * SS * CP;
  static_assert(OC % 8 == 0, "s2d channels must fill 16-B chunks");
  const long total = (long)N * Ho * Wo;
  for (long pix = (long)blockIdx.x * kT + threadIdx.x; pix < total; pix += (long)gridDim.x * kT) {
    const int j = (int)(pix % Wo);
    const long t = pix / Wo;
    const int i = (int)(t % Ho);
    const int n = (int)(t / Ho);
    bf16_t v[OC];
#pragma unroll
    for (int a = 0; a < SS; ++a) {
      const int h = SS * i + a - pad;
#pragma unroll
      for (int b = 0; b < SS; ++b) {
        const int w = SS * j + b - pad;
        const bool in = h >= 0 && h < H && w >= 0 && w < W;
        const bf16_t* src = x + (((long)n * H + (in ? h : 0)) * W + (in ? w : 0)) * C;
#pragma unroll
        for (int ch = 0; ch < CP; ++ch) v[(a * SS + b) * CP + ch] = (in && ch < C) ? src[ch] : (bf16_t)0;
      }
    }
    uint4* dst = reinterpret_cast<uint4*>(xs + pix * OC);
#pragma unroll
    for (int k = 0; k < OC / 8; ++k) {
      uint4 u;
      u.x = (uint32_t)v[8 * k + 0] | ((uint32_t)v[8 * k + 1] << 16);
      u.y = (uint32_t)v[8 * k + 2] | ((uint32_t)v[8 * k + 3] << 16);
      u.z = (uint32_t)v[8 * k + 4] | ((uint32_t)v[8 * k + 5] << 16);
      u.w = (uint32_t)v[8 * k + 6] | ((uint32_t)v[8 * k + 7] << 16);
      dst[k] = u;
    }
  }
}

// Row form for images whose rows are whole 16-B chunks (the 224 x 224 x 3 ResNet input: 1344 B
// per row): a block stages one output row's SS input rows in LDS with 16-B loads -- the pixel
// kernel above issues 12 two-byte loads per output pixel (~3.3 TB/s at b1984) -- then every lane
// assembles one output pixel's channels from LDS and stores them as 16-B chunks.  Same values,
// same zero fill: bit-identical.
constexpr int kS2dT = 128, kS2dMaxChunks = 256;   // input rows of up to 2048 bf16
template <int SS, int CP>
__global__ void __launch_bounds__(kS2dT)
s2d_rows_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xs, int N, int H, int W,
                int C, int Ho, int Wo, int pad) {
  constexpr int OC = SS * SS * CP;
  static_assert(OC % 8 == 0, "s2d channels must fill 16-B chunks");
  __shared__ uint4 rows[SS][kS2dMaxChunks];
  const int rc = W * C / 8;                        // 16-B chunks per input row (host-checked)
  const long nrows = (long)N * Ho;
  const bf16_t* rb = reinterpret_cast<const bf16_t*>(&rows[0][0]);
  for (long r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int i = (int)(r % Ho);
    const int n = (int)(r / Ho);
    __syncthreads();                               // the previous row's LDS reads are done
#pragma unroll
    for (int a = 0; a < SS; ++a) {
      const int h = SS * i + a - pad;
      const bool in = h >= 0 && h < H;
      const uint4* src = reinterpret_cast<const uint4*>(x + ((long)n * H + (in ? h : 0)) * W * C);
      for (int k = threadIdx.x; k < rc; k += kS2dT) rows[a][k] = in ? src[k] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < Wo; j += kS2dT) {
      bf16_t v[OC];
#pragma unroll
      for (int a = 0; a < SS; ++a)
#pragma unroll
        for (int b = 0; b < SS; ++b) {
          const int w = SS * j + b - pad;
          const bool in = w >= 0 && w < W;
          const bf16_t* src = rb + a * kS2dMaxChunks * 8 + (in ? w : 0) * C;
#pragma unroll
          for (int ch = 0; ch < CP; ++ch) v[(a * SS + b) * CP + ch] = (in && ch < C) ? src[ch] : (bf16_t)0;
        }
      uint4* dst = reinterpret_cast<uint4*>(xs + (r * Wo + j) * OC);
#pragma unroll
      for (int k = 0; k < OC / 8; ++k) {
        uint4 u;
        u.x = (uint32_t)v[8 * k + 0] | ((uint32_t)v[8 * k + 1] << 16);
        u.y = (uint32_t)v[8 * k + 2] | ((uint32_t)v[8 * k + 3] << 16);
        u.z = (uint32_t)v[8 * k + 4] | ((uint32_t)v[8 * k + 5] << 16);
        u.w = (uint32_t)v[8 * k + 6] | ((uint32_t)v[8 * k + 7] << 16);
        dst[k] = u;
      }
    }
  }
}

}  // namespace

void dtf_maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* arg, int N, int H, int W, int C,
                     int P, int Q, int kh, int kw, int sh, int sw, int ph, int pw,
                     hipStream_t st) {
  const long total = (long)N * P * Q * (C / 8);
  if (total < (1L << 31))
    hipLaunchKernelGGL(maxpool_fwd_kernel<uint32_t>, dim3(grid_for(total)), dim3(kT), 0, st, x, y,
                       arg, N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<uint64_t>, dim3(grid_for(total)), dim3(kT), 0, st, x, y,
                       arg, N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
}

static int g_pool_blocked = 1;   // 0: always the generic gather (tests compare both)
void dtf_pool_set_blocked(int v) { g_pool_blocked = v; }

void dtf_maxpool_bwd(const bf16_t* dy, const uint8_t* arg, bf16_t* dx, int N, int H, int W,
                     int C, int P, int Q, int kh, int kw, int sh, int sw, int ph, int pw,
                     hipStream_t st) {
  const long total = (long)N * H * W * (C / 8);
  if (g_pool_blocked && kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 &&
      P == (H - 1) / 2 + 1 && Q == (W - 1) / 2 + 1 && total < (1L << 31))
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel, dim3(grid_for(total / 4 + 1)), dim3(kT), 0, st, dy,
                       arg, dx, N, H, W, C, P, Q);
  else if (total < (1L << 31))
    hipLaunchKernelGGL(maxpool_bwd_kernel<uint32_t>, dim3(grid_for(total)), dim3(kT), 0, st, dy,
                       arg, dx, N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<uint64_t>, dim3(grid_for(total)), dim3(kT), 0, st, dy,
                       arg, dx, N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
}

void dtf_gap_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st) {
  const long total = (long)N * (C / 8);
  hipLaunchKernelGGL(gap_fwd_kernel, dim3((int)((total + kT - 1) / kT)), dim3(kT), 0, st, x, y, N,
                     HW, C);
}

void dtf_gap_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(grid_for((long)N * HW * (C / 8))), dim3(kT), 0, st, dy,
                     dx, N, HW, C);
}

static int g_s2d_rows = 1;   // 0: always the per-pixel kernel (tests compare both)
void dtf_s2d_set_rows(int v) { g_s2d_rows = v; }

void dtf_s2d_input(const bf16_t* x, bf16_t* xs, int N, int H, int W, int C, int Ho, int Wo,
                   int s, int cp, int pad, hipStream_t st) {
  if (s != 2 || (cp != 2 && cp != 4) || C > cp)
    throw std::runtime_error("s2d_input: stride 2 with C <= 4 channels only (image stems)");
  // row form: whole 16-B input rows that fit the LDS image, 16-B aligned input
  if (g_s2d_rows && (W * C) % 8 == 0 && W * C / 8 <= kS2dMaxChunks &&
      (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const long nrows = (long)N * Ho;
    const int gr = (int)(nrows < 16384 ? nrows : 16384);
    if (cp == 4)
      hipLaunchKernelGGL((s2d_rows_kernel<2, 4>), dim3(gr), dim3(kS2dT), 0, st, x, xs, N, H, W, C,
                         Ho, Wo, pad);
    else
      hipLaunchKernelGGL((s2d_rows_kernel<2, 2>), dim3(gr), dim3(kS2dT), 0, st, x, xs, N, H, W, C,
                         Ho, Wo, pad);
    return;
  }
  const long total = (long)N * Ho * Wo;
  long g = (total + kT - 1) / kT;
  if (g > 65536) g = 65536;
  if (cp == 4)
    hipLaunchKernelGGL((s2d_input_kernel<2, 4>), dim3((int)g), dim3(kT), 0, st, x, xs, N, H, W, C,
                       Ho, Wo, pad);
  else
    hipLaunchKernelGGL((s2d_input_kernel<2, 2>), dim3((int)g), dim3(kT), 0, st, x, xs, N, H, W, C,
                       Ho, Wo, pad);
}

void dtf_bn_relu_maxpool_fwd(const bf16_t* x, const float* scale, const float* shift, bf16_t* y,
                             uint8_t* arg, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                             int sh, int sw, int ph, int pw, hipStream_t st) {
  if (C % 8) throw std::runtime_error("bn_relu_maxpool: C % 8 != 0");
  if (kh * kw > 255) throw std::runtime_error("bn_relu_maxpool: window too large");
  const long total = (long)N * P * Q * (C / 8);
  if (g_pool_blocked && kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 &&
      kT % (C / 8) == 0 && (long)N * H * W * (C / 8) < 2147483647L)
    hipLaunchKernelGGL(bn_relu_maxpool3s2_fwd_kernel, dim3(grid_for(total)), dim3(kT), 0, st, x,
                       scale, shift, y, arg, N, H, W, C, P, Q);
  else if (total < 2147483647L && (long)N * H * W * C < 2147483647L)
    hipLaunchKernelGGL(bn_relu_maxpool_fwd_kernel<uint32_t>, dim3(grid_for(total)), dim3(kT), 0,
                       st, x, scale, shift, y, arg, N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  else
    hipLaunchKernelGGL(bn_relu_maxpool_fwd_kernel<uint64_t>, dim3(grid_for(total)), dim3(kT), 0,
                       st, x, scale, shift, y, arg, N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
}

// grid caps of the stem pool + BN backward passes (reduce, apply): the reduce at 1024 blocks
// left a third of a round (147 VGPRs: 3 blocks per CU) -- 996 -> 921 us at 4096 on the b1984 stem
// (profiles/measurements/r5_pool_bwd_grid_probe.jsonl)
static int g_pool_bwd_cap[2] = {4096, 4096};
void dtf_pool_bn_bwd_set_caps(int reduce_cap, int apply_cap) {
  if (reduce_cap > 0) g_pool_bwd_cap[0] = reduce_cap;
  if (apply_cap > 0) g_pool_bwd_cap[1] = apply_cap;
}
int dtf_pool_bn_bwd_blocks(int N, int H, int W, int C) {
  const long total = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  long g = (total + kT - 1) / kT;
  if (g > g_pool_bwd_cap[0]) g = g_pool_bwd_cap[0];
  return (int)(g < 1 ? 1 : g);
}

static void pool_bn_check(int N, int H, int W, int C, int P, int Q) {
  // 16-B-chunk indices are 32-bit in the kernel
  if (C % 8 || kT % (C / 8) || P != (H - 1) / 2 + 1 || Q != (W - 1) / 2 + 1 ||
      (long)N * H * W * (C / 8) >= 2147483647L)
    throw std::runtime_error("pool3s2_bn_bwd: unsupported shape");
}

void dtf_pool_bn_bwd_reduce(const bf16_t* dy, const uint8_t* arg, const bf16_t* x,
                            const float* mean, const float* invstd, const float* fsc,
                            const float* fsh, float* partial, int N, int H, int W, int C, int P,
                            int Q, hipStream_t st) {
  pool_bn_check(N, H, W, C, P, Q);
  hipLaunchKernelGGL(pool3s2_bn_bwd_kernel<false>, dim3(dtf_pool_bn_bwd_blocks(N, H, W, C)),
                     dim3(kT), 0, st, dy, arg, x, mean, invstd, nullptr, fsc, fsh, nullptr,
                     partial, N, H, W, C, P, Q);
}

void dtf_pool_bn_bwd_apply(const bf16_t* dy, const uint8_t* arg, const bf16_t* x, const float* cA,
                           const float* cB, const float* cC, const float* fsc, const float* fsh,
                           bf16_t* dx, int N, int H, int W, int C, int P, int Q, hipStream_t st) {
  pool_bn_check(N, H, W, C, P, Q);
  const long total = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  long ga = (total + kT - 1) / kT;
  if (ga > g_pool_bwd_cap[1]) ga = g_pool_bwd_cap[1];
  hipLaunchKernelGGL(pool3s2_bn_bwd_kernel<true>, dim3((unsigned)(ga < 1 ? 1 : ga)), dim3(kT), 0, st, dy, arg,
                     x, cA, cB, cC, fsc, fsh, dx, nullptr, N, H, W, C, P, Q);
}
