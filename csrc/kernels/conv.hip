// Implicit-GEMM convolution on MFMA (gfx950), NHWC bf16, fp32 accumulate.
//
//   Y[m, k] = sum_{t, c} X[n(m), h(m,t), w(m,t), c] * Wt[k, t*C + c]
//
// "Tap table" formulation: an output grid (N, P, Q) and a list of T taps (dh_t, dw_t); output
// pixel (n,p,q) reads input pixel (p*sh + dh_t, q*sw + dw_t) for tap t (zero outside the image)
// and is stored at Y[n, p*osh + oh0, q*osw + ow0, :] of an [N, Ho, Wo, Kout] tensor.
//   * forward:              taps = {(r - pad_h, s - pad_w)}, (osh,osw,oh0,ow0) = (1,1,0,0)
//   * data-grad, stride 1:  forward conv of dY with the C<->K transposed filter and
//                           taps {(pad_h - r, pad_w - s)}
//   * data-grad, stride s:  one launch per output phase class (a, b) in [0,s)^2 with the taps
//                           that hit that class; osh = osw = s, (oh0, ow0) = (a, b)
// so one MFMA kernel serves SURVEY.md K3/K5/N-K1 forward and dgrad.
//
// Tiling (cdna_hip_programming.md §5, 2-stage pipeline):
//   block = 256 threads = 4 waves in WAVES_M x WAVES_N, wave tile 64x64 built from 4x4
//   v_mfma_f32_16x16x32_bf16 tiles (16x16x32 holds a higher clock than 32x32x16 under load:
//   MI355X_MICROARCH.md "DVFS give-back" (7)).
//   K-step BK = 64 (C % 64 == 0) or 32 (C % 32 == 0); each (row, tap) supplies BK contiguous
//   channels = one 128-B / 64-B line per output row, loaded 16 B per lane.
//   Loads are raw BUFFER loads (guide §5.5 T8): the per-lane byte offset of a padding tap is set
//   out of range, so the hardware range check returns zeros — zero padding with no branches.
//   Register staging with the T14 split: next tile's global loads are issued before the MFMAs
//   of the current tile and written to the other LDS buffer after them; one barrier per K-step.
//   LDS rows are XOR-swizzled by 16-B chunk so ds_read_b128 fragment reads of 16 different rows
//   are conflict-free (T2).
//   Epilogue: accumulators -> bf16 -> LDS -> 16-B coalesced global stores.
//   Tile order: XCD-aware bijective remap of the block id, N-tile fastest so blocks sharing an
//   A panel run on the same XCD's L2 (T1).
//   GATHER (template): 0 = each K-step lies inside one tap (C % BK == 0: every ResNet body conv);
//   2 = per-16-B-chunk taps from an LDS copy of the table (C % 8 == 0: the stem / MNIST conv1 after
//   their input channels are zero-padded to 8 by the host); 1 = per-element gather (any C).
//   The tap table arrives as a kernel argument; it is only ever read with wave-uniform indices
//   (scalar loads) — per-lane indices go through a copy in LDS.
#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"

#define DTF_MAX_TAPS 64

struct TapTable {
  int n;
  int dh[DTF_MAX_TAPS];
  int dw[DTF_MAX_TAPS];
};

struct ConvGeom {
  int N, H, W, C;        // input
  int P, Q;              // output grid of this launch
  int sh, sw;            // input stride
  int Kout;              // output channels (GEMM N)
  int Kpad;              // filter row stride (T*C rounded up to BK)
  int Ho, Wo;            // output tensor spatial dims
  int osh, osw, oh0, ow0;// output placement
  int acc;               // 1: Y += result (dgrad accumulating onto a residual gradient)
                         // 2: Y = result + acc_src * relu_mask (see acc_add8)
  const bf16_t* acc_src; // acc 2: the residual BN's incoming dy, [N, Ho, Wo, Kout] like Y
  const uint8_t* acc_mask;  // acc 2: that BN's forward ReLU bit mask (1 byte per 8 channels)
  const float* bias;        // fused epilogue (register kernel only): Y = act(conv + bias[k])
  int relu;                 //   tf.layers.conv2d(activation=tf.nn.relu) -- MNIST K3/K5
  int nt;                   // non-temporal output stores (set by dtf_conv_igemm)
  // BN + ReLU on load (halo kernels, forward): X is a BatchNorm INPUT; the kernel normalises its
  // patch in LDS with y = bf16(max(x * lsc[c] + lsh[c], 0)) -- the apply pass's arithmetic -- and
  // writes the rows it owns to ly (the weight gradient's operand), so the apply pass never runs
  const float* lsc;
  const float* lsh;
  bf16_t* ly;
};

// Residual-gradient accumulation in the dgrad epilogue.  acc 1 reads the materialised residual
// gradient back from Y; acc 2 forms it on the fly as dy * relu_mask from the residual BN's own
// inputs, so that BN's backward never writes it (saves one full-tensor write per identity block;
// bit-identical: the masked copy is exact).
DTF_DEV uint4 acc_add8(const ConvGeom& g, const bf16_t* Y, long off, uint4 v) {
  float a[8], b[8];
  unpack8(v, a);
  if (g.acc == 2) {
    unpack8(*reinterpret_cast<const uint4*>(g.acc_src + off), b);
    const uint32_t m = g.acc_mask[off >> 3];
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = (m >> e) & 1u ? b[e] : 0.f;
  } else {
    unpack8(*reinterpret_cast<const uint4*>(Y + off), b);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] += b[e];
  return pack8(a);
}

// Fused BatchNorm-backward statistics in the DATA-GRADIENT epilogue: when this launch produces
// dy of a training-mode BN's output (the BN sits right before this conv in the forward pass), the
// epilogue also accumulates, per channel, sum(dz) and sum(dz * (x - mean) * invstd) with
// dz = dy * relu_mask(x) -- exactly bn_reduce_kernel<1>'s sums, from the bf16-ROUNDED final dy
// (after a fused residual accumulation) -- into row `row0 + tile` of a [rows][2][Kout] slab the
// BN's finalize combines.  Saves the backward reduce pass its full re-read of dy.
// bit 0: one LDS stage when the whole reduction is one K-step; bit 1: BK 32 for 1x1 convs with
// C <= 128; bit 2: BK 32 for every 1x1; bit 3: BK 32 for every register-kernel conv; bit 4:
// the <= 128-VGPR (4 waves/SIMD) build of the BK-32 kernels (see dtf_conv_igemm)
static int g_small_k = 31;  // bits 0-4: same-box A/B +2.4 % (bit 2), +2.0 % (bit 4), +0.5 % (bit 3)

struct BnBwdEpi {
  const bf16_t* x;          // BN input, same [N, Ho, Wo, Kout] layout as Y
  const float* mean;
  const float* invstd;
  const float* fsc;         // forward scale / shift (mask recomputed from x, mkind 2)
  const float* fsh;
  const uint8_t* mask;      // ReLU bit mask (mkind 1)
  float* part;              // null: off
  int mkind;                // 0 no ReLU, 1 bit mask, 2 from x
  int row0;
};

namespace {

constexpr int kThreads = 256;

DTF_DEV void load8(const float* __restrict__ p, int c, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p + c);
  const float4 b = *reinterpret_cast<const float4*>(p + c + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// per-thread BN-backward partial sums of one 8-channel column chunk
struct BnbAcc {
  float s0[8], s1[8], mu[8], is[8], sc[8], sh[8];
  DTF_DEV void init(const BnBwdEpi& e, int c, bool ok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) { s0[i] = 0.f; s1[i] = 0.f; mu[i] = 0.f; is[i] = 0.f; sc[i] = 0.f; sh[i] = 0.f; }
    if (!ok) return;
    load8(e.mean, c, mu);
    load8(e.invstd, c, is);
    if (e.mkind == 2) { load8(e.fsc, c, sc); load8(e.fsh, c, sh); }
  }
  DTF_DEV void add(const BnBwdEpi& e, long off, const uint4& v) {
    float g[8], xv[8];
    unpack8(v, g);
    unpack8(*reinterpret_cast<const uint4*>(e.x + off), xv);
    if (e.mkind == 1) {
      const uint32_t mb = e.mask[off >> 3];
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = (mb >> i) & 1u ? g[i] : 0.f;
    } else if (e.mkind == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = __builtin_fmaf(xv[i], sc[i], sh[i]) > 0.f ? g[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) { s0[i] += g[i]; s1[i] += g[i] * (xv[i] - mu[i]) * is[i]; }
  }
  // same, with x (and the mask byte) already in registers (prefetched before the LDS staging)
  DTF_DEV void add_pre(const BnBwdEpi& e, const uint4& v, const uint4& xr, uint32_t mb) {
    float g[8], xv[8];
    unpack8(v, g);
    unpack8(xr, xv);
    if (e.mkind == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = (mb >> i) & 1u ? g[i] : 0.f;
    } else if (e.mkind == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = __builtin_fmaf(xv[i], sc[i], sh[i]) > 0.f ? g[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) { s0[i] += g[i]; s1[i] += g[i] * (xv[i] - mu[i]) * is[i]; }
  }
  // red: [orows][2][BN] floats; fixed-order column sums -> slab row
  template <int BN, int NT>
  DTF_DEV void flush(const BnBwdEpi& e, float* red, int orow, int oc, int orows, int tid, int tm,
                     int n0, int Kout) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[(orow * 2 + 0) * BN + oc * 8 + i] = s0[i];
      red[(orow * 2 + 1) * BN + oc * 8 + i] = s1[i];
    }
    // LDS visibility only: a __syncthreads() would also drain vmcnt, i.e. wait for the tile's
    // output stores issued just before
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    for (int idx = tid; idx < 2 * BN; idx += NT) {
      const int which = idx / BN, col = idx % BN;
      if (n0 + col >= Kout) continue;
      float t = 0.f;
      for (int k = 0; k < orows; ++k) t += red[(k * 2 + which) * BN + col];
      e.part[((long)(e.row0 + tm) * 2 + which) * Kout + n0 + col] = t;
    }
  }
};
constexpr uint32_t kOOB = 0xFFFFFFF0u;   // byte offset the buffer range check always rejects

template <int BK>
DTF_DEV int swz_chunk(int row, int chunk) {
  constexpr int CPR = BK / 8;           // 16-B chunks per row
  constexpr int RPB = 16 / CPR;         // rows per 256-B bank row
  return chunk ^ ((row / RPB) % CPR);
}

DTF_DEV __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
DTF_DEV uint4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
DTF_DEV uint32_t bload2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}

// HI_OCC (BK 32, g_small_k bit 4): ask for <= 128 VGPRs -> 4 waves/SIMD, so the 35-KB-LDS 1x1
// launches can run 4 blocks per CU instead of 3
// STATS: the launch fuses the BatchNorm statistics (stats != nullptr); a template flag so the
// launches without them (data gradients) keep their register budget
// The kernel body, for tile `bid` of the launch's (tiles_m x tiles_n) grid; TT: the tap table
// type (TapTable, or the grouped launch's per-class TapTableG)
template <int WAVES_M, int WAVES_N, int BK, int GATHER, bool BNB, bool STATS, class TT>
DTF_DEV __attribute__((always_inline)) void
conv_igemm_body(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                bf16_t* __restrict__ Y, const ConvGeom& g, const TT& taps,
                float* __restrict__ stats, const BnBwdEpi& bnb, const int bid) {
  constexpr int BM = 64 * WAVES_M, BN = 64 * WAVES_N;
  constexpr int CPR = BK / 8;                            // chunks per row
  constexpr int A_CHUNKS = BM * CPR / kThreads;          // 16-B loads per thread for A
  constexpr int B_CHUNKS = BN * CPR / kThreads;
  constexpr int ROWS_PER_PASS = kThreads / CPR;
  constexpr int STAGE_ELEMS = (BM + BN) * BK;            // bf16 elements per LDS stage
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  int* lds_taps = reinterpret_cast<int*>(lds + 2 * STAGE_ELEMS);   // [2][DTF_MAX_TAPS]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;

  const int M = g.N * g.P * g.Q;
  const int tiles_n = (g.Kout + BN - 1) / BN;
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM;
  const int n0 = tn * BN;

  const int K = taps.n * g.C;
  const int nk = (K + BK - 1) / BK;
  // X descriptor based at the first image this tile's rows touch (64-bit pointer math): the
  // 32-bit buffer offsets then span a few images only, so no tensor-size limit remains
  const int PQ = g.P * g.Q;
  const int n_lo = m0 / PQ;
  const int n_hi = min(g.N - 1, (min(m0 + BM, M) - 1) / PQ);
  const long img = (long)g.H * g.W * g.C;
  const auto rx = rsrc(X + n_lo * img, (uint32_t)((n_hi - n_lo + 1) * img * 2));
  const auto rw = rsrc(Wt, (uint32_t)g.Kout * g.Kpad * 2u);

  if constexpr (GATHER != 0) {
    if (tid == 0)
      for (int t = 0; t < taps.n; ++t) { lds_taps[t] = taps.dh[t]; lds_taps[DTF_MAX_TAPS + t] = taps.dw[t]; }
  }

  // ---- per-thread A rows: decode (n, p, q) once (32-bit; host guarantees M < 2^31)
  const int chunk = tid % CPR;
  int a_pix[A_CHUNKS], a_h[A_CHUNKS], a_w[A_CHUNKS];
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) {
    const int m = m0 + tid / CPR + i * ROWS_PER_PASS;
    const bool ok = m < M;
    const int mm = ok ? m : 0;
    const int q = mm % g.Q;
    const int t = mm / g.Q;
    const int p = t % g.P;
    const int n = t / g.P;
    a_pix[i] = (n - n_lo) * g.H * g.W;        // image base pixel (relative to the descriptor)
    a_h[i] = ok ? p * g.sh : -(1 << 24);      // invalid rows fail every bounds test
    a_w[i] = q * g.sw;
  }

  uint4 ra[A_CHUNKS], rb[B_CHUNKS];

  auto load_stage = [&](int kt) {
    const int k0 = kt * BK;
    if constexpr (GATHER == 0) {
      const int t = __builtin_amdgcn_readfirstlane(k0 / g.C);
      const int c0 = k0 - t * g.C + chunk * 8;
      const int dh = taps.dh[t], dw = taps.dw[t];          // uniform index: scalar loads
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        const int h = a_h[i] + dh, w = a_w[i] + dw;
        const bool ok = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
        const uint32_t off = ok ? (uint32_t)(((a_pix[i] + h * g.W + w) * g.C + c0) * 2) : kOOB;
        ra[i] = bload16(rx, off);
      }
    } else if constexpr (GATHER == 2) {
      const int k = k0 + chunk * 8;                   // 8 channels of one tap per 16-B chunk
      const int t = k / g.C, c = k - t * g.C;
      const int tt = k < K ? t : 0;
      const int dh = lds_taps[tt], dw = lds_taps[DTF_MAX_TAPS + tt];
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        const int h = a_h[i] + dh, w = a_w[i] + dw;
        const bool ok = k < K && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
        ra[i] = bload16(rx, ok ? (uint32_t)(((a_pix[i] + h * g.W + w) * g.C + c) * 2) : kOOB);
      }
    } else {
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        uint32_t wv[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          uint32_t pair = 0;
#pragma unroll
          for (int e1 = 0; e1 < 2; ++e1) {
            const int k = k0 + chunk * 8 + e2 * 2 + e1;
            const int t = k / g.C, c = k - t * g.C;
            const int tt = t < taps.n ? t : 0;
            const int h = a_h[i] + lds_taps[tt], w = a_w[i] + lds_taps[DTF_MAX_TAPS + tt];
            const bool ok = k < K && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
            const uint32_t off = ok ? (uint32_t)(((a_pix[i] + h * g.W + w) * g.C + c) * 2) : kOOB;
            pair |= bload2(rx, off) << (16 * e1);
          }
          wv[e2] = pair;
        }
        ra[i] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
    }
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) {
      const int nrow = n0 + tid / CPR + i * ROWS_PER_PASS;
      const uint32_t off = nrow < g.Kout ? (uint32_t)((nrow * g.Kpad + k0 + chunk * 8) * 2) : kOOB;
      rb[i] = bload16(rw, off);
    }
  };

  auto store_stage = [&](int buf) {
    bf16_t* sa = lds + buf * STAGE_ELEMS;
    bf16_t* sb = sa + BM * BK;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int r = tid / CPR + i * ROWS_PER_PASS;
      *reinterpret_cast<uint4*>(sa + r * BK + swz_chunk<BK>(r, chunk) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) {
      const int r = tid / CPR + i * ROWS_PER_PASS;
      *reinterpret_cast<uint4*>(sb + r * BK + swz_chunk<BK>(r, chunk) * 8) = rb[i];
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  if constexpr (GATHER != 0) __syncthreads();   // tap table visible before the first gather
  load_stage(0);
  store_stage(0);
  __syncthreads();

  const int frow = lane & 15, fq = lane >> 4;
  // Epilogue rows are decoded up front and, for the fused BN-backward sums, the BN input x (+ mask
  // bytes) of every row this thread will store is loaded during the LAST K-step: those HBM reads
  // overlap its MFMAs and the LDS staging instead of stalling the store loop.  The barriers from
  // there to the store loop are raw s_barriers behind lgkmcnt(0) (a __syncthreads() would drain
  // vmcnt, i.e. wait for the prefetch).
  constexpr int OCPR = BN / 8;                 // 16-B chunks per output row
  constexpr int OROWS = kThreads / OCPR;
  constexpr int NR = BM / OROWS;               // rows per thread
  const int oc = tid % OCPR;
  const bool col_ok = n0 + oc * 8 < g.Kout;
  // output element offset of this thread's k-th epilogue row (-1: none); 64-bit
  auto row_off = [&](int k) -> long {
    const int m = m0 + tid / OCPR + k * OROWS;
    const int q = m % g.Q;
    const int t = m / g.Q;
    const int p = t % g.P;
    const int n = t / g.P;
    const int ho = p * g.osh + g.oh0, wo = q * g.osw + g.ow0;
    return (m < M && col_ok) ? (((long)n * g.Ho + ho) * g.Wo + wo) * g.Kout + n0 + oc * 8 : -1;
  };
  long offs[NR];
  uint4 xpre[BNB ? NR : 1];
  uint32_t mpre[BNB ? (NR + 3) / 4 : 1];       // the rows' mask bytes, 4 per register
  auto prefetch_epilogue = [&]() {
#pragma unroll
    for (int k = 0; k < NR; ++k) offs[k] = row_off(k);
#pragma unroll
    for (int k = 0; k < (NR + 3) / 4; ++k) mpre[k] = 0u;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      xpre[k] = offs[k] >= 0 ? *reinterpret_cast<const uint4*>(bnb.x + offs[k]) : make_uint4(0, 0, 0, 0);
      if (offs[k] >= 0 && bnb.mkind == 1) mpre[k >> 2] |= (uint32_t)bnb.mask[offs[k] >> 3] << (8 * (k & 3));
    }
  };
  if constexpr (BNB) { if (nk == 0) prefetch_epilogue(); }

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_stage(kt + 1);
    else if constexpr (BNB) prefetch_epilogue();
    const bf16_t* sa = lds + cur * STAGE_ELEMS;
    const bf16_t* sb = sa + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t af[4], bfr[4];
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8_t*>(sa + r * BK + swz_chunk<BK>(r, ch) * 8);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 64 + j * 16 + frow;
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(sb + r * BK + swz_chunk<BK>(r, ch) * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      store_stage(cur ^ 1);
      __syncthreads();
    }
  }
  if constexpr (!BNB) {
#pragma unroll
    for (int k = 0; k < NR; ++k) offs[k] = row_off(k);
  }
  // every wave is done reading the last stage before the staging below overwrites it
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();

  // (explicit wait states between the MFMA chain and the first consumer of its results)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  constexpr int LDC = BN + 8;
  bf16_t* st = lds;
  float bj[4] = {0.f, 0.f, 0.f, 0.f};
  if (g.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + j * 16 + frow;
      bj[j] = col < g.Kout ? g.bias[col] : 0.f;
    }
  }
  // Fused BatchNorm statistics (training forward) from the registers: per output channel, the
  // sum and sum of squares of this tile's bf16-ROUNDED outputs (exactly what the BN will
  // normalise).  Each lane sums its column over its 16 rows, the 4 lane groups sharing a column
  // combine by cross-lane adds, and the WAVES_M waves of a column meet in LDS; thread `col`
  // writes row `tm` of the [tiles_m][2][Kout] slab that the BN finalize combines in a fixed
  // order.  (The earlier pass over the staged tile cost 64 dependent 2-byte LDS reads per thread
  // in the epilogue of every tile.)
  constexpr bool do_stats = STATS;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + fq * 4 + r;
        const int col = wn * 64 + j * 16 + frow;
        float v = acc[i][j][r] + bj[j];
        if (g.relu) v = fmaxf(v, 0.f);
        const bf16_t h = f2bf(v);
        st[row * LDC + col] = h;
        if (do_stats && m0 + row < M) {
          const float q = bf2f(h);
          s1[j] += q;
          s2[j] += q * q;
        }
      }
  float* red = reinterpret_cast<float*>(st + BM * LDC);   // [WAVES_M][2][BN], past the tile
  if (do_stats) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    if (fq == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + frow;
        red[(wm * 2 + 0) * BN + col] = s1[j];
        red[(wm * 2 + 1) * BN + col] = s2[j];
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  if (do_stats && tid < BN && n0 + tid < g.Kout) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < WAVES_M; ++k) { a += red[(k * 2 + 0) * BN + tid]; b += red[(k * 2 + 1) * BN + tid]; }
    stats[((long)tm * 2 + 0) * g.Kout + n0 + tid] = a;
    stats[((long)tm * 2 + 1) * g.Kout + n0 + tid] = b;
  }
  BnbAcc ba;
  if constexpr (BNB) ba.init(bnb, n0 + oc * 8, col_ok);
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    if (offs[k] < 0) continue;
    const int r = tid / OCPR + k * OROWS;
    const long off = offs[k];
    uint4 v = *reinterpret_cast<const uint4*>(st + r * LDC + oc * 8);
    // fused residual-gradient add: one extra 16-B read instead of an add kernel
    if (g.acc) v = acc_add8(g, Y, off, v);
    st16(Y + off, v, g.nt);
    if constexpr (BNB) ba.add_pre(bnb, v, xpre[k], (mpre[k >> 2] >> (8 * (k & 3))) & 0xFFu);
  }
  if constexpr (BNB)
    ba.template flush<BN, kThreads>(bnb, reinterpret_cast<float*>(st + BM * LDC), tid / OCPR, oc,
                                    OROWS, tid, tm, n0, g.Kout);
}

template <int WAVES_M, int WAVES_N, int BK, int GATHER, bool BNB, bool HI_OCC = false,
          bool STATS = false>
__global__ void __launch_bounds__(kThreads, HI_OCC ? 4 : 2)
conv_igemm_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                  bf16_t* __restrict__ Y, const ConvGeom g, const TapTable taps,
                  float* __restrict__ stats, const BnBwdEpi bnb) {
  constexpr int BM = 64 * WAVES_M, BN = 64 * WAVES_N;
  const int nwg = ((g.N * g.P * g.Q + BM - 1) / BM) * ((g.Kout + BN - 1) / BN);
  conv_igemm_body<WAVES_M, WAVES_N, BK, GATHER, BNB, STATS>(X, Wt, Y, g, taps, stats, bnb,
                                                            xcd_remap(blockIdx.x, nwg));
}

// ---------------------------------------------------------------------------------------------
// Grouped strided data gradient: the s x s output phase classes of a stride-s conv's dgrad
// (conv2d_dgrad: one dense stride-1 sub-convolution per class, over that class's taps only --
// no zero taps) in ONE launch instead of one per class.  Per class, only the output placement
// (oh0, ow0), the tap list, the filter slice and the BN-backward slab rows differ; every class
// has the same tile count (the host requires it), and blocks are interleaved class-fastest, so
// the classes of one M-tile run side by side and share its dY rows in L2: 1.00 vs 1.15 ms for
// the 56x56x128 stride-2 layer at b1984 (class-major in one grid: 1.26 ms; tools/conv_gap.py).
constexpr int kGrpMax = 4;
constexpr int kGrpTaps = 9;
struct TapTableG {
  int n;
  int dh[kGrpTaps];
  int dw[kGrpTaps];
};
struct ConvGroup {
  int n;                               // classes
  // per class: the whole geometry / epilogue record, read in place from the kernel arguments
  // (a copy with the class's fields patched in costs registers the BN-sum epilogue needs)
  const bf16_t* Wt[kGrpMax];           // [Kout][Kpad] per class
  ConvGeom g[kGrpMax];
  BnBwdEpi bnb[kGrpMax];
  TapTableG taps[kGrpMax];
};

template <int WAVES_M, int WAVES_N, bool BNB, bool HI_OCC>
__global__ void __launch_bounds__(kThreads, HI_OCC ? 4 : 2)
conv_igemm_grouped_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                          const ConvGroup grp) {
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int cls = __builtin_amdgcn_readfirstlane(b % grp.n);      // classes interleaved per tile
  const int tile = b / grp.n;
  conv_igemm_body<WAVES_M, WAVES_N, 32, 0, BNB, false>(X, grp.Wt[cls], Y, grp.g[cls],
                                                      grp.taps[cls], nullptr, grp.bnb[cls], tile);
}

template <int WM, int WN, int BK, int GEN>
void launch_cfg(const bf16_t* X, const bf16_t* Wt, bf16_t* Y, const ConvGeom& g,
                const TapTable& taps, float* stats, const BnBwdEpi& bnb, hipStream_t st) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int OROWS = kThreads / (BN / 8);
  const long M = (long)g.N * g.P * g.Q;
  const long tiles = ((M + BM - 1) / BM) * ((g.Kout + BN - 1) / BN);
  // one K-step (1x1 convs with C <= BK, the stage-1 layers): only stage 0 is ever filled, so size
  // the LDS for one stage -> 3 blocks/CU (VGPR-bound) instead of 2 on these latency-bound shapes
  const int nk = (taps.n * g.C + BK - 1) / BK;
  const size_t stage = (size_t)(BM + BN) * BK * sizeof(bf16_t) *
                           ((nk > 1 || GEN != 0 || !(g_small_k & 1)) ? 2 : 1) +
                       2 * DTF_MAX_TAPS * sizeof(int);
  const size_t scratch = bnb.part ? (size_t)OROWS * 2 * BN : (size_t)2 * kThreads;
  const size_t epi = (size_t)BM * (BN + 8) * sizeof(bf16_t) +
                    scratch * sizeof(float);          // + stats / BN-backward reduction scratch
  const size_t lds = stage > epi ? stage : epi;
  if (bnb.part) {
    if constexpr (GEN == 0)
      hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, BK, GEN, true>), dim3((unsigned)tiles),
                         dim3(kThreads), lds, st, X, Wt, Y, g, taps, stats, bnb);
    else
      throw std::runtime_error("conv: fused BN-backward sums need a C % 32 == 0 dgrad");
  } else if (BK == 32 && GEN == 0 && (g_small_k & 16)) {
    if (stats)
      hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, BK, GEN, false, BK == 32 && GEN == 0, true>),
                         dim3((unsigned)tiles), dim3(kThreads), lds, st, X, Wt, Y, g, taps, stats, bnb);
    else
      hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, BK, GEN, false, BK == 32 && GEN == 0>),
                         dim3((unsigned)tiles), dim3(kThreads), lds, st, X, Wt, Y, g, taps, stats, bnb);
  } else {
    if (stats)
      hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, BK, GEN, false, false, true>),
                         dim3((unsigned)tiles), dim3(kThreads), lds, st, X, Wt, Y, g, taps, stats, bnb);
    else
      hipLaunchKernelGGL((conv_igemm_kernel<WM, WN, BK, GEN, false>), dim3((unsigned)tiles),
                         dim3(kThreads), lds, st, X, Wt, Y, g, taps, stats, bnb);
  }
}

// ---------------------------------------------------------------------------------------------
// 8-wave LDS-DMA variant (GATHER 0, BK 64): 256 x 128 tile, waves 4 (M) x 2 (N) of 64 x 64,
// THREE LDS stages filled by `buffer_load_dwordx4 ... lds` (no staging VGPRs, no ds_write pass),
// loads issued two K-steps ahead (cdna_hip_programming.md §5 "glds vs register staging", 3-buffer
// row: counted vmcnt + raw s_barrier, never __syncthreads() inside the loop).  One block per CU
// (144 KB of LDS), 2 waves per SIMD.  The DMA writes each wave-instruction's 64 x 16 B
// lane-linearly, so the XOR chunk swizzle of the fragment reads is applied on the SOURCE side:
// LDS slot s of row r receives source chunk s ^ ((r >> 1) & 7).  Padding taps get an
// out-of-range buffer offset -> the hardware range check delivers zeros.
constexpr int kDmaThreads = 512;
constexpr int kDmaBM = 256, kDmaBN = 128, kDmaBK = 64;
constexpr int kDmaA = kDmaBM * kDmaBK;                    // A elements per stage
constexpr int kDmaStage = (kDmaBM + kDmaBN) * kDmaBK;     // 24576 bf16 = 48 KB
template <bool BNB>
__global__ void __launch_bounds__(kDmaThreads, 1)
conv_igemm_dma_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                      bf16_t* __restrict__ Y, const ConvGeom g, const TapTable taps,
                      float* __restrict__ stats, const BnBwdEpi bnb) {
  __shared__ __attribute__((aligned(16))) bf16_t lds[3 * kDmaStage];
  bf16_t* const s0 = lds;
  bf16_t* const s1 = lds + kDmaStage;
  bf16_t* const s2 = lds + 2 * kDmaStage;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int M = g.N * g.P * g.Q;
  const int tiles_n = (g.Kout + kDmaBN - 1) / kDmaBN;
  const int tiles_m = (M + kDmaBM - 1) / kDmaBM;
  const int bid = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * kDmaBM, n0 = tn * kDmaBN;
  const int nk = taps.n * g.C / kDmaBK;
  const int PQ = g.P * g.Q;                          // descriptor rebased per tile (see above)
  const int n_lo = m0 / PQ;
  const int n_hi = min(g.N - 1, (min(m0 + kDmaBM, M) - 1) / PQ);
  const long img = (long)g.H * g.W * g.C;
  const i32x4_t rx = rsrc_quad(X + n_lo * img, (uint32_t)((n_hi - n_lo + 1) * img * 2));
  const i32x4_t rw = rsrc_quad(Wt, (uint32_t)g.Kout * g.Kpad * 2u);
  const uint32_t lds0 = lds_addr(lds);

  // this wave fills row-groups (8 rows x 128 B = 1 KB) wave + 8j of each stage's 48 groups:
  // j = 0..3 -> A rows, j = 4, 5 -> B rows.  Lane -> (row lrow of the group, LDS slot).
  const int lrow = lane >> 3, slot = lane & 7;
  int a_pix[4], a_h[4], a_w[4], a_ch[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (wave + 8 * j) + lrow;
    const int m = m0 + row;
    const bool ok = m < M;
    const int mm = ok ? m : 0;
    const int q = mm % g.Q;
    const int t = mm / g.Q;
    const int p = t % g.P;
    const int n = t / g.P;
    a_pix[j] = (n - n_lo) * g.H * g.W;
    a_h[j] = ok ? p * g.sh : -(1 << 24);
    a_w[j] = q * g.sw;
    a_ch[j] = (slot ^ ((row >> 1) & 7)) * 8;
  }
  int b_off[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (wave + 8 * j) + lrow;
    const int nrow = n0 + row;
    b_off[j] = nrow < g.Kout ? nrow * g.Kpad + (slot ^ ((row >> 1) & 7)) * 8 : -1;
  }

  // K-step kt >= nk is issued too, with every lane out of range (no memory traffic): each step
  // then has exactly 6 DMAs per wave in flight behind it, so the wait count is a constant
  auto issue = [&](int kt, int stage) {
    const bool live = kt < nk;
    const int k0 = (live ? kt : 0) * kDmaBK;
    const int t = __builtin_amdgcn_readfirstlane(k0 / g.C);
    const int c0 = k0 - t * g.C;
    const int dh = taps.dh[t], dw = taps.dw[t];
    const uint32_t base = lds0 + (uint32_t)(stage * kDmaStage + wave * 512) * 2u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = a_h[j] + dh, w = a_w[j] + dw;
      const bool ok = live && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      const uint32_t off = ok ? (uint32_t)(((a_pix[j] + h * g.W + w) * g.C + c0 + a_ch[j]) * 2) : kOOB;
      dma16(rx, base + j * 8 * 1024, off);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t off = (live && b_off[j] >= 0) ? (uint32_t)((b_off[j] + k0) * 2) : kOOB;
      dma16(rw, base + kDmaA * 2 + j * 8 * 1024, off);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fq = lane >> 4;
  auto compute = [&](const bf16_t* sa) {
    const bf16_t* sb = sa + kDmaA;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t af[4], bfr[4];
      const int ch = ks * 4 + fq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + frow;
        af[i] = *reinterpret_cast<const bf16x8_t*>(sa + r * kDmaBK + swz_chunk<kDmaBK>(r, ch) * 8);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 64 + j * 16 + frow;
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(sb + r * kDmaBK + swz_chunk<kDmaBK>(r, ch) * 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // step k: own DMAs of step k done (step k+1's 6 may still fly) -> barrier (every wave's step-k
  // data landed AND every wave finished step k-1, freeing its stage) -> issue k+2 into that
  // stage -> MFMAs on step k.
  issue(0, 0);
  issue(1, 1);
  int cur = 0, nxt = 2;
  for (int kt = 0; kt < nk; ++kt) {
    DTF_WAIT_VM(6);
    raw_barrier();
    issue(kt + 2, nxt);
    compute(lds + cur * kDmaStage);
    cur = cur == 2 ? 0 : cur + 1;
    nxt = nxt == 2 ? 0 : nxt + 1;
  }

  // ---- epilogue (as conv_igemm_kernel): rows 0..127 of the tile staged in s0, 128..255 in s1
  constexpr int OCPR = kDmaBN / 8;
  constexpr int OROWS = kDmaThreads / OCPR;
  constexpr int NR = kDmaBM / OROWS;
  const int oc = tid % OCPR;
  const bool col_ok = n0 + oc * 8 < g.Kout;
  long offs[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const int m = m0 + tid / OCPR + k * OROWS;
    const int q = m % g.Q;
    const int t = m / g.Q;
    const int p = t % g.P;
    const int n = t / g.P;
    const int ho = p * g.osh + g.oh0, wo = q * g.osw + g.ow0;
    offs[k] = (m < M && col_ok) ? (((long)n * g.Ho + ho) * g.Wo + wo) * g.Kout + n0 + oc * 8 : -1;
  }
  uint4 xpre[BNB ? NR : 1];
  uint32_t mpre[BNB ? NR : 1];
  DTF_WAIT_VM(0);              // the trailing (out-of-range) DMAs still target the LDS stages
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  if constexpr (BNB) {         // BN input rows in flight while the tile is staged
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      xpre[k] = offs[k] >= 0 ? *reinterpret_cast<const uint4*>(bnb.x + offs[k]) : make_uint4(0, 0, 0, 0);
      mpre[k] = (offs[k] >= 0 && bnb.mkind == 1) ? (uint32_t)bnb.mask[offs[k] >> 3] : 0u;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  constexpr int LDC = kDmaBN + 8;
  {
    bf16_t* st = wm < 2 ? s0 : s1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = (wm & 1) * 64 + i * 16 + fq * 4 + r;
          const int col = wn * 64 + j * 16 + frow;
          st[row * LDC + col] = f2bf(acc[i][j][r]);
        }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  BnbAcc ba;
  if constexpr (BNB) ba.init(bnb, n0 + oc * 8, col_ok);
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    if (offs[k] < 0) continue;
    const int r = tid / OCPR + k * OROWS;
    const long off = offs[k];
    const bf16_t* st = r < 128 ? s0 : s1;
    uint4 v = *reinterpret_cast<const uint4*>(st + (r & 127) * LDC + oc * 8);
    if (g.acc) v = acc_add8(g, Y, off, v);
    st16(Y + off, v, g.nt);
    if constexpr (BNB) ba.add_pre(bnb, v, xpre[k], mpre[k]);
  }
  if constexpr (BNB)   // [32][2][128] floats = 32 KB in the third stage buffer
    ba.template flush<kDmaBN, kDmaThreads>(bnb, reinterpret_cast<float*>(s2), tid / OCPR, oc,
                                           OROWS, tid, tm, n0, g.Kout);
  if (stats) {   // fused BN partial sums, same contract as conv_igemm_kernel (row tm of the slab)
    constexpr int GROUPS = kDmaThreads / kDmaBN;     // 4 groups of 64 rows
    constexpr int RPG = kDmaBM / GROUPS;
    float* red = reinterpret_cast<float*>(s2);
    const int col = tid % kDmaBN, grp = tid / kDmaBN;
    const bf16_t* st = grp < 2 ? s0 : s1;
    float a1 = 0.f, a2 = 0.f;
    const int rend = min(RPG * (grp + 1), M - m0);
    for (int r = RPG * grp; r < rend; ++r) {
      const float v = bf2f(st[(r & 127) * LDC + col]);
      a1 += v;
      a2 += v * v;
    }
    red[(grp * 2 + 0) * kDmaBN + col] = a1;
    red[(grp * 2 + 1) * kDmaBN + col] = a2;
    __syncthreads();
    if (grp == 0 && n0 + col < g.Kout) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) { a += red[(k * 2 + 0) * kDmaBN + col]; b += red[(k * 2 + 1) * kDmaBN + col]; }
      stats[((long)tm * 2 + 0) * g.Kout + n0 + col] = a;
      stats[((long)tm * 2 + 1) * g.Kout + n0 + col] = b;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Halo-tiled 3x3 stride-1 conv for the 56 x 56 x 64 -> 64 layers (stage 1 c2 forward AND its data
// gradient, which is the same conv with flipped taps).  The implicit-GEMM kernels re-fetch every
// input pixel once per tap (9x) through L2 and run these K=64-channel layers at ~0.14 of the MFMA
// roof; here a block owns 4 full output rows of one image (224 pixels x 64 channels), loads the
// 6 x 58-pixel input patch ONCE into LDS by LDS-DMA (zero halo from the buffer range check) and
// reads all 9 taps' A fragments from it; the 9 per-tap 64 x 64 filter slices stream through a
// double-buffered LDS ring (8 KB each).  4 waves as 2 (M: 7 fragments = 112 px) x 2 (N: 32).
// LDS rows are 128 B (64 bf16) with the chunk XOR swizzle of swz_chunk<64> by row (patch pixel
// index / filter row), applied on the DMA source side.
constexpr int kHaloTH = 4;        // output rows per block (whole image rows)
#ifndef DTF_HALO_FREG_D1
#define DTF_HALO_FREG_D1 2        // FREG register-ring depth, 56 x 56 x 64 family (steps)
#endif
#ifndef DTF_HALO_FREG_D2
#define DTF_HALO_FREG_D2 3        // FREG register-ring depth, 28 x 28 x 128 family (steps)
#endif

// C: input channels (64 | 128), W: image width (56 | 28), WMW x (4 / WMW) waves, NT output
// channels per block.  7 x 2 MFMA fragments per wave in both families:
//   56 x 56 x 64  -> 64 : M 224 = 2 waves x 7 frags, NT 64  = 2 waves x 2 frags
//   28 x 28 x 128 -> 128: M 112 = 1 wave  x 7 frags, NT 128 = 4 waves x 2 frags
template <int C, int W, int WMW, int NT>
struct HaloCfg {
  static constexpr int PW = W + 2;                       // patch width (pixels)
  static constexpr int PIX = (kHaloTH + 2) * PW;         // patch pixels
  static constexpr int ROWB = C * 2;                     // bytes per patch pixel
  static constexpr int PPI = 1024 / ROWB;                // pixels per 1-KB DMA
  static constexpr int PIXAL = (PIX + PPI - 1) / PPI * PPI;
  static constexpr int M = kHaloTH * W;                  // output pixels per block
  static constexpr int WNW = 4 / WMW;
  static constexpr int MF = M / 16 / WMW;                // M fragments per wave
  static constexpr int NF = NT / WNW / 16;               // N fragments per wave
  static constexpr int KS = C / 64;                      // 64-channel slices per tap
  static constexpr int WST = NT * 64;                    // filter elements per stage
  static constexpr int LDC = NT + 8;
  static constexpr size_t LDS = (size_t)(PIXAL * C + 2 * WST) * 2;
  static constexpr size_t lds(int st, int nstg = 2) {
    return (size_t)(st * PIXAL * C + nstg * WST) * 2;
  }
  static constexpr size_t LDS_FREG = (size_t)PIXAL * C * 2;    // FREG: the patch only
  static_assert(M % (16 * WMW) == 0 && NT % (16 * WNW) == 0, "halo tiling");
  static_assert((size_t)M * LDC * 2 + (size_t)2 * NT * (kThreads / NT) * 4 <= (size_t)PIXAL * C * 2,
                "halo epilogue must fit in the patch region");
};

// chunk swizzle of a patch pixel row, keyed by u = prow * W + pcol (the pixel index WITHOUT the
// two halo columns per row, so a fragment's 16 output pixels are 16 consecutive u for every tap,
// across output-row boundaries too).  ds_read_b128 serves a wave in four 16-lane groups
// ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, +32; MI355X_MICROARCH.md "LDS"): half of a group
// reads chunk c of 8 consecutive-u pixels, the other half chunk c ^ 1 of the 8 next.  An EVEN
// swizzle value keeps the halves apart (bit 0 of the chunk) and 4 (128-B rows: two pixels per
// bank row) / 8 (256-B rows) distinct values per half cover the rest: conflict-free for any u
// offset.  (Keyed by the padded index with (p >> 1) & 7 / p & 15, the reads were ~1.7-way
// conflicted: SQ_LDS_BANK_CONFLICT ~ SQ_BUSY_CYCLES on both families.)
template <int C>
DTF_DEV int halo_swz(int u) { return C == 64 ? (((u >> 1) & 3) << 1) : ((u & 7) << 1); }

// ST strips per block (ST x 4 waves): the per-tap filter slices stream through LDS once per
// block, so two strips per block halve the filter's L2 -> LDS traffic.  Measured no faster at
// b2048 (one 8-wave block per CU instead of two 4-wave blocks: the blocks' barrier phases no
// longer overlap; profiles/measurements/r2_halo_strips_ab_b2048.txt), so ST = 1 by default.
//
// FREG: the filter never enters LDS.  Each wave streams its own B fragments (its NF x 16 output
// channels x 64 input channels per step) from L2 straight into VGPRs, D steps ahead of the MFMAs
// that use them (a register ring), so the K loop has no barrier and no per-step wait on a DMA that
// was issued only one step earlier (~190 ns of MFMA cover against an L2 round trip several times
// that).  LDS holds only the patch: 44-46 KB per block instead of 60-78 KB, which leaves room for
// a third block per CU.  The MFMA order is unchanged, so the outputs are bit-identical.
//
// BNB (a data gradient whose output feeds a BatchNorm(+ReLU) backward -- the c2 data gradient of a
// bottleneck, consumed by BN1): the epilogue also forms that BN's backward partial sums
// (sum dz, sum dz * xhat, dz = dy masked by the forward ReLU) per output channel, one slab row
// per block (BnbAcc, the contract of conv_igemm_kernel's BNB epilogue).  The BN input x is loaded
// for the thread's output rows before the tile is staged, so its latency hides under the staging.
// NSTG: filter-slice ring depth (LDS stages; the slice of step s + NSTG - 1 is issued at step s,
// so a slice has NSTG - 1 steps of MFMA work to arrive from L2; 2 = the original double buffer)
// BNLP (timing probe only, y not written): the BN-on-load forward without its y stores
template <int C, int W, int WMW, int NT, int ST = 1, bool FREG = false, bool BNB = false,
          int NSTG = 2, bool BNL = false, int BNLP = 0>
__global__ void __launch_bounds__(kThreads * ST, ST == 1 ? 2 : 1)
conv3x3_halo_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                    bf16_t* __restrict__ Y, const ConvGeom g, const TapTable taps,
                    float* __restrict__ stats, const BnBwdEpi bnb) {
  using H = HaloCfg<C, W, WMW, NT>;
  static_assert(!BNL || (!FREG && ST == 1 && !BNB), "BN on load: the forward ring kernel");
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int tid = threadIdx.x & (kThreads - 1), lane = tid & 63;   // tid within the strip
  const int wall = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int sid = wall >> 2, wave = wall & 3;                    // strip, wave within the strip
  bf16_t* const patch = lds + sid * (H::PIXAL * C);              // [ST][PIXAL][C]
  bf16_t* const wst = lds + ST * (H::PIXAL * C);                 // [NSTG][NT][64]
  // BNL: per 8-channel chunk {scale[8], shift[8]} (16 floats), past the filter ring
  float* const bnl_prm = reinterpret_cast<float*>(wst + NSTG * H::WST);
  if constexpr (BNL) {
    for (int t = tid; t < C / 4; t += kThreads) {       // float4 t: channels 4t .. 4t + 3
      const int ch = t >> 1, half = t & 1;
      reinterpret_cast<float4*>(bnl_prm)[ch * 4 + half] =
          *reinterpret_cast<const float4*>(g.lsc + 4 * t);
      reinterpret_cast<float4*>(bnl_prm)[ch * 4 + 2 + half] =
          *reinterpret_cast<const float4*>(g.lsh + 4 * t);
    }
  }
  const int wm = wave / H::WNW, wn = wave % H::WNW;
  const int tiles_h = g.H / kHaloTH;
  const int tm = blockIdx.x * ST + sid;                          // (image, row-tile)
  const bool live = tm < g.N * tiles_h;                          // odd tail: a dead strip
  const int n = live ? tm / tiles_h : 0, h0 = live ? (tm % tiles_h) * kHaloTH : 0;
  const int n0 = blockIdx.y * NT;                                // output-channel tile
  const i32x4_t rx = rsrc_quad(X + (long)n * g.H * g.W * g.C, (uint32_t)g.H * g.W * g.C * 2u);
  const i32x4_t rw = rsrc_quad(Wt, (uint32_t)g.Kout * g.Kpad * 2u);
  const uint32_t lds_patch = lds_addr(patch), lds_w = lds_addr(wst);

  // ---- patch: whole 1-KB DMAs of PPI pixels; wave w issues q = w, w + 4, ...
  {
    constexpr int CPP = H::ROWB / 16;                            // chunks per pixel
    const int lp = lane / CPP, slot = lane % CPP;
    for (int q = wave; q < H::PIXAL / H::PPI; q += 4) {
      const int pix = q * H::PPI + lp;
      const int pr = pix / H::PW, pc = pix - pr * H::PW;
      const int h = h0 - 1 + pr, w = pc - 1;
      const int chunk = slot ^ halo_swz<C>(pr * W + pc);
      const bool ok = live && pix < H::PIX && (unsigned)h < (unsigned)g.H &&
                      (unsigned)w < (unsigned)g.W;
      const uint32_t off = ok ? (uint32_t)(((h * g.W + w) * C + chunk * 8) * 2) : kOOB;
      dma16(rx, lds_patch + (uint32_t)q * 1024u, off);
    }
  }
  // ---- BNB: this thread's epilogue rows of the BN input x (and mask bytes), loaded now -- the
  // block runs at most two waves per SIMD (LDS-bound), so the 28 registers are free, and the loads
  // complete under the main loop instead of in front of the epilogue's stores
  constexpr int OCPR = NT / 8;
  constexpr int OROWS = kThreads / OCPR;                         // rows per store pass
  constexpr int NR = H::M / OROWS;                               // store passes
  static_assert(H::M % OROWS == 0, "halo epilogue rows");
  const long ybase = ((long)n * g.H + h0) * g.W;                 // first output pixel of the tile
  const int oc = tid % OCPR;
  const bool col_ok = n0 + oc * 8 < g.Kout;
  uint4 xpre[BNB ? NR : 1];
  uint32_t mpre[BNB ? NR : 1];
  if constexpr (BNB) {
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const long off = (ybase + tid / OCPR + k * OROWS) * g.Kout + n0 + oc * 8;
      const bool ok = live && col_ok;
      xpre[k] = ok ? *reinterpret_cast<const uint4*>(bnb.x + off) : make_uint4(0, 0, 0, 0);
      mpre[k] = (ok && bnb.mkind == 1) ? (uint32_t)bnb.mask[off >> 3] : 0u;
    }
  }
  // ---- filter slice of step (tap t, channel slice s): NT rows x 64 channels (128-B rows)
  const int lp8 = lane >> 3, slot8 = lane & 7;
  auto issue_w = [&](int step, int stage) {
    const int t = step / H::KS, s = step - t * H::KS;
#pragma unroll
    for (int i = 0; i < NT / (32 * ST); ++i) {
      const int q = wall + 4 * ST * i;
      const int row = q * 8 + lp8;
      const int chunk = slot8 ^ ((row >> 1) & 7);
      const int kr = n0 + row;
      const uint32_t off = (t < taps.n && kr < g.Kout)
                               ? (uint32_t)((kr * g.Kpad + t * C + s * 64 + chunk * 8) * 2) : kOOB;
      dma16(rw, lds_w + (uint32_t)(stage * H::WST) * 2u + (uint32_t)q * 1024u, off);
    }
  };
  if constexpr (!FREG) {
#pragma unroll
    for (int s0 = 0; s0 < NSTG - 1; ++s0) issue_w(s0, s0);
  }
  // DMA instructions per wave per filter slice: the slices younger than the one a step reads
  constexpr int kDPW = NT / (32 * ST);
  constexpr int kYoung = (NSTG - 2) * kDPW;
  static_assert(kYoung <= 4 || kYoung == 6 || kYoung == 8, "halo ring: add the wait count");

  // per-lane A rows: output pixel m = wm * (MF * 16) + 16 i + frow -> patch pixel of tap (0, 0)
  const int frow = lane & 15, fq = lane >> 4;
  int pbase[H::MF], ubase[H::MF];     // patch index and its halo-free twin (swizzle key)
#pragma unroll
  for (int i = 0; i < H::MF; ++i) {
    const int m = wm * (H::MF * 16) + 16 * i + frow;
    const int orow = m / W, ocol = m - orow * W;
    pbase[i] = (orow + 1) * H::PW + ocol + 1;
    ubase[i] = (orow + 1) * W + ocol + 1;
  }
  f32x4_t acc[H::MF][H::NF];
#pragma unroll
  for (int i = 0; i < H::MF; ++i)
#pragma unroll
    for (int j = 0; j < H::NF; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  if constexpr (FREG) {
    static_assert(ST == 1, "FREG: one strip per block");
    constexpr int NSTEP = 9 * H::KS;                 // halo_family() admits 9-tap convs only
    constexpr int D = H::KS == 2 ? DTF_HALO_FREG_D2 : DTF_HALO_FREG_D1;   // ring depth (steps)
    const bf16_t* wr[H::NF];
#pragma unroll
    for (int j = 0; j < H::NF; ++j)
      wr[j] = Wt + (long)(n0 + wn * (H::NF * 16) + 16 * j + frow) * g.Kpad + fq * 8;
    bf16x8_t bq[D][2][H::NF];
    auto ldB = [&](int step, bf16x8_t (&b)[2][H::NF]) {
      const int t = step / H::KS, s = step - t * H::KS;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < H::NF; ++j)
          b[ks][j] = *reinterpret_cast<const bf16x8_t*>(wr[j] + t * C + s * 64 + ks * 32);
    };
#pragma unroll
    for (int p = 0; p < D; ++p) ldB(p, bq[p]);
    // the patch DMAs were issued before these D * 2 * NF loads: waiting until only those are
    // outstanding means this wave's patch pieces have landed; the barrier covers everyone's
    static_assert(D * 2 * H::NF <= 40 && D * 2 * H::NF % 4 == 0, "add the wait count");
    if constexpr (D * 2 * H::NF == 8) DTF_WAIT_VM(8);
    else if constexpr (D * 2 * H::NF == 12) DTF_WAIT_VM(12);
    else if constexpr (D * 2 * H::NF == 16) DTF_WAIT_VM(16);
    else if constexpr (D * 2 * H::NF == 20) DTF_WAIT_VM(20);
    else if constexpr (D * 2 * H::NF == 24) DTF_WAIT_VM(24);
    else if constexpr (D * 2 * H::NF == 28) DTF_WAIT_VM(28);
    else if constexpr (D * 2 * H::NF == 32) DTF_WAIT_VM(32);
    else if constexpr (D * 2 * H::NF == 36) DTF_WAIT_VM(36);
    else DTF_WAIT_VM(40);
    __syncthreads();
#pragma unroll
    for (int step = 0; step < NSTEP; ++step) {
      const int t = step / H::KS, s = step - t * H::KS;
      const int dpix = taps.dh[t] * H::PW + taps.dw[t];
      const int dupix = taps.dh[t] * W + taps.dw[t];
      bf16x8_t (&cur)[2][H::NF] = bq[step % D];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int pch = s * 8 + ks * 4 + fq;
#pragma unroll
        for (int i = 0; i < H::MF; ++i) {
          const int p = pbase[i] + dpix;
          const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(
              patch + p * C + ((pch ^ halo_swz<C>(ubase[i] + dupix)) << 3));
#pragma unroll
          for (int j = 0; j < H::NF; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, cur[ks][j], acc[i][j], 0, 0, 0);
        }
      }
      // refill the slot this step consumed; the scheduling fences keep the loads here (left
      // alone, the compiler sinks them next to their use and the ring degenerates to vmcnt(1-3))
      __builtin_amdgcn_sched_barrier(0);
      if (step + D < NSTEP) ldB(step + D, cur);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
  const int nsteps = taps.n * H::KS;
  for (int step = 0; step < nsteps; ++step) {
    // patch (step 0) and this step's filter slice landed (own DMAs; the kYoung younger slice
    // DMAs may fly) ...
    if constexpr (kYoung == 0) DTF_WAIT_VM(0);
    else if constexpr (kYoung == 1) DTF_WAIT_VM(1);
    else if constexpr (kYoung == 2) DTF_WAIT_VM(2);
    else if constexpr (kYoung == 3) DTF_WAIT_VM(3);
    else if constexpr (kYoung == 4) DTF_WAIT_VM(4);
    else if constexpr (kYoung == 6) DTF_WAIT_VM(6);
    else DTF_WAIT_VM(8);
    __syncthreads();           // ... everyone's; everyone done reading the slot restaged next
    if constexpr (BNL) {
      if (step == 0) {
        // BN + ReLU of the landed patch, in place (padding pixels stay zero); the rows this block
        // owns (input rows h0 .. h0 + TH - 1, every pixel exactly once over the grid) go to ly.
        // Fully unrolled over the thread's items (the patch reads and the per-chunk scale / shift
        // reads from the LDS copy all issue ahead of their use)
        constexpr int CPP = H::ROWB / 16;
        constexpr int ITEMS = (H::PIX * CPP + kThreads - 1) / kThreads;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
          const int idx = tid + k * kThreads;
          const int pix = idx / CPP, slot = idx - pix * CPP;
          const int pr = pix / H::PW, pc = pix - pr * H::PW;
          const int h = h0 - 1 + pr, w = pc - 1;
          if (idx >= H::PIX * CPP || (unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W)
            continue;
          const int lch = slot ^ halo_swz<C>(pr * W + pc);      // logical chunk in this slot
          uint4* pp = reinterpret_cast<uint4*>(patch + pix * C + slot * 8);
          const float4* sp = reinterpret_cast<const float4*>(bnl_prm + lch * 16);
          const float4 s0 = sp[0], s1 = sp[1], t0 = sp[2], t1 = sp[3];
          const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          const float sf[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
          float v[8];
          unpack8(*pp, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(__builtin_fmaf(v[e], sc[e], sf[e]), 0.f);
          const uint4 pk = pack8(v);
          *pp = pk;
          if (BNLP == 0 && pr >= 1 && pr <= kHaloTH)
            *reinterpret_cast<uint4*>(g.ly + (((long)n * g.H + h) * g.W + w) * C + lch * 8) = pk;
        }
        __syncthreads();
      }
    }
    // past the last step: out-of-range, no traffic
    issue_w(step + NSTG - 1, (step + NSTG - 1) % NSTG);
    const int t = step / H::KS, s = step - t * H::KS;
    const int dpix = taps.dh[t] * H::PW + taps.dw[t];            // wave-uniform
    const int dupix = taps.dh[t] * W + taps.dw[t];
    const bf16_t* sw = wst + (step % NSTG) * H::WST;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fq;                                // chunk within the 64-ch slice
      bf16x8_t bfr[H::NF];
#pragma unroll
      for (int j = 0; j < H::NF; ++j) {
        const int r = wn * (H::NF * 16) + 16 * j + frow;
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(sw + r * 64 + ((ch ^ ((r >> 1) & 7)) << 3));
      }
      const int pch = s * 8 + ch;                                // chunk within the pixel row
#pragma unroll
      for (int i = 0; i < H::MF; ++i) {
        const int p = pbase[i] + dpix;
        const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(
            patch + p * C + ((pch ^ halo_swz<C>(ubase[i] + dupix)) << 3));
#pragma unroll
        for (int j = 0; j < H::NF; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  }
  DTF_WAIT_VM(0);
  __syncthreads();
  // ---- epilogue: bf16 tile [M][NT + 8] in LDS (over the patch) -> 16-B stores; BN partials
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  constexpr int LDC = H::LDC;
  bf16_t* st = patch;
#pragma unroll
  for (int i = 0; i < H::MF; ++i)
#pragma unroll
    for (int j = 0; j < H::NF; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        st[(wm * (H::MF * 16) + 16 * i + fq * 4 + r) * LDC + wn * (H::NF * 16) + 16 * j + frow] =
            f2bf(acc[i][j][r]);
  __syncthreads();
  BnbAcc ba;
  if constexpr (BNB) ba.init(bnb, n0 + oc * 8, col_ok);
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const int r = tid / OCPR + k * OROWS;
    if (!col_ok || !live) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(st + r * LDC + oc * 8);
    st16(Y + (ybase + r) * g.Kout + n0 + oc * 8, v, g.nt);
    if constexpr (BNB) ba.add_pre(bnb, v, xpre[k], mpre[k]);
  }
  if constexpr (BNB) {
    // dead strips (odd tail) add nothing but still write their (zero) slab row: every row of the
    // slab the BN finalize sums is defined
    ba.template flush<NT, kThreads>(bnb, reinterpret_cast<float*>(st + H::M * LDC), tid / OCPR,
                                    oc, OROWS, tid, tm, n0, g.Kout);
  }
  // per-channel sum / sum of squares of the rounded outputs -> slab row tm: a column pass over the
  // staged tile.  (Summing the stored 16-B values in the store loop and folding the lanes by
  // shuffles -- as the stem kernel below now does -- measured 10-45 us SLOWER per call here in the
  // network, profiles/r6; register sums from the accumulators were slower in round 2.)
  if (stats) {
    constexpr int GROUPS = kThreads / NT;
    constexpr int RPG = H::M / GROUPS;
    float* red = reinterpret_cast<float*>(st + H::M * LDC);      // [GROUPS][2][NT]
    const int col = tid % NT, grp = tid / NT;
    float a1 = 0.f, a2 = 0.f;
    for (int r = grp * RPG; r < (grp + 1) * RPG; ++r) {
      const float v = bf2f(st[r * LDC + col]);
      a1 += v;
      a2 += v * v;
    }
    red[(grp * 2 + 0) * NT + col] = a1;
    red[(grp * 2 + 1) * NT + col] = a2;
    __syncthreads();
    if (grp == 0 && n0 + col < g.Kout && live) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) { a += red[(k * 2 + 0) * NT + col]; b += red[(k * 2 + 1) * NT + col]; }
      stats[((long)tm * 2 + 0) * g.Kout + n0 + col] = a;
      stats[((long)tm * 2 + 1) * g.Kout + n0 + col] = b;
    }
  }
}


// ---------------------------------------------------------------------------------------------
// ResNet stem as a halo conv: the 7x7/2 conv on the 3-channel image runs as a 4x4 stride-1 conv
// over the 2x2 space-to-depth image (16 channels, [N][P+3][Q+3][16], padding already applied).
// The register kernel's chunk gather re-reads each input pixel from L2 for all 16 taps (~0.5 KB
// of L2 traffic per output pixel) and ran at ~0.35 of its roof.  Here a block owns kStemTH whole
// output rows of one image: the kStemTH + 3 input rows it needs are ONE contiguous span of
// global memory, copied into LDS by lane-linear LDS-DMA, and the full 64 x 256 filter sits in
// LDS (row pitch padded to 528 B: conflict-free fragment reads); every tap is then an LDS read.
// K order = tap-major, channel-minor (the filter layout [64][4][4][16]): one 32-deep K-step is
// taps (r, s), (r, s + 1) of one row -- 64 contiguous patch bytes -- so each A fragment is a
// single 16-B LDS read.  Epilogue as the 3x3 halo kernel (bf16 tile through LDS, 16-B stores,
// BatchNorm partial sums of the rounded outputs, one slab row per block).  Same MFMA chain
// order as the register kernel (K in order, 32 at a time): bit-identical outputs.
constexpr int kStemTH = 4;                 // output rows per block
constexpr int kStemC = 16, kStemK = 64, kStemKD = 256;
constexpr int kStemWP = kStemKD + 8;       // filter LDS row pitch (elements)

template <int Q>
struct StemCfg {
  static constexpr int PW = Q + 3;                                // s2d row width (pixels)
  static constexpr int PATCH = (kStemTH + 3) * PW * kStemC;       // elements
  static constexpr int PATCH_DMA = (PATCH * 2 + 1023) / 1024;     // 1-KB DMA instructions
  static constexpr int PATCH_AL = PATCH_DMA * 512;                // elements (DMA-rounded)
  static constexpr int M = kStemTH * Q;                           // output pixels per block
  static constexpr int MF = M / 16 / 4;                           // M fragments per wave
  static constexpr int LDC = kStemK + 8;
  static constexpr size_t MAIN = ((size_t)PATCH_AL + (size_t)kStemK * kStemWP) * 2;
  static constexpr size_t EPI = (size_t)M * LDC * 2 + (size_t)2 * kStemK * (kThreads / kStemK) * 4;
  static constexpr size_t LDS = MAIN > EPI ? MAIN : EPI;
  static_assert(M % 64 == 0, "stem tiling: 4 waves x 16-row fragments");
};

template <int Q>
__global__ void __launch_bounds__(kThreads, 2)
conv_stem_halo_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                      bf16_t* __restrict__ Y, const ConvGeom g, float* __restrict__ stats) {
  using H = StemCfg<Q>;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  bf16_t* const patch = lds;                                      // [(TH+3) * PW][16]
  bf16_t* const wl = lds + H::PATCH_AL;                           // [64][kStemWP]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_h = g.P / kStemTH;
  const int tm = blockIdx.x;
  const int n = tm / tiles_h, p0 = (tm % tiles_h) * kStemTH;
  // ---- patch: input rows p0 .. p0 + TH + 2 of image n, one contiguous span
  {
    const long base = ((long)n * g.H + p0) * g.W * kStemC;        // elements
    const i32x4_t rx = rsrc_quad(X + base, (uint32_t)(H::PATCH * 2));
    const uint32_t lp = lds_addr(patch);
    for (int q = wave; q < H::PATCH_DMA; q += 4)
      dma16(rx, lp + (uint32_t)q * 1024u, (uint32_t)(q * 1024 + lane * 16));   // tail: OOB -> 0
  }
  // ---- filter [64][256] -> padded LDS rows (16-B loads + ds_write; L2-resident after block 0)
  for (int c = tid; c < kStemK * kStemKD / 8; c += kThreads) {
    const int row = c / (kStemKD / 8), ch = c % (kStemKD / 8);
    *reinterpret_cast<uint4*>(wl + row * kStemWP + ch * 8) =
        *reinterpret_cast<const uint4*>(Wt + (long)row * g.Kpad + ch * 8);
  }
  DTF_WAIT_VM(0);
  __syncthreads();

  const int frow = lane & 15, fq = lane >> 4;
  int pb[H::MF];                                                  // patch pixel of tap (0, 0)
#pragma unroll
  for (int i = 0; i < H::MF; ++i) {
    const int m = wave * (H::MF * 16) + 16 * i + frow;
    const int orow = m / Q, ocol = m - orow * Q;
    pb[i] = orow * H::PW + ocol;
  }
  f32x4_t acc[H::MF][4];
#pragma unroll
  for (int i = 0; i < H::MF; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int kc = 0; kc < kStemKD / 32; ++kc) {
    const int r = kc >> 1, sc = (kc & 1) * 2;                    // taps (r, sc), (r, sc + 1)
    const int dpix = r * H::PW + sc;
    bf16x8_t bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8_t*>(wl + (16 * j + frow) * kStemWP + kc * 32 + fq * 8);
#pragma unroll
    for (int i = 0; i < H::MF; ++i) {
      const bf16x8_t af =
          *reinterpret_cast<const bf16x8_t*>(patch + (pb[i] + dpix) * kStemC + fq * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();
  // ---- epilogue: bf16 tile [M][64 + 8] in LDS -> 16-B stores; BN partials of the rounded values
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  constexpr int LDC = H::LDC;
  bf16_t* st = lds;
#pragma unroll
  for (int i = 0; i < H::MF; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        st[(wave * (H::MF * 16) + 16 * i + fq * 4 + rr) * LDC + 16 * j + frow] = f2bf(acc[i][j][rr]);
  __syncthreads();
  const long ybase = ((long)n * g.P + p0) * Q;
  constexpr int OCPR = kStemK / 8;
  const int oc = tid % OCPR;
  // BN statistics summed from the stored 16-B values as they pass (see conv3x3_halo_kernel)
  float q1[8], q2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { q1[e] = 0.f; q2[e] = 0.f; }
  static_assert(H::M % (kThreads / OCPR) == 0, "stem epilogue rows");
#pragma unroll
  for (int k = 0; k < H::M / (kThreads / OCPR); ++k) {
    const int rr = tid / OCPR + k * (kThreads / OCPR);
    const uint4 v = *reinterpret_cast<const uint4*>(st + rr * LDC + oc * 8);
    st16(Y + (ybase + rr) * kStemK + oc * 8, v, g.nt);
    if (stats) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) { q1[e] += f[e]; q2[e] = __builtin_fmaf(f[e], f[e], q2[e]); }
    }
  }
  if (stats) {
#pragma unroll
    for (int msk = OCPR; msk < 64; msk <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        q1[e] += __shfl_xor(q1[e], msk, 64);
        q2[e] += __shfl_xor(q2[e], msk, 64);
      }
    float* red = reinterpret_cast<float*>(st + H::M * LDC);       // [4 waves][2][64]
    if (lane < OCPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 2 + 0) * kStemK + oc * 8 + e] = q1[e];
        red[(wave * 2 + 1) * kStemK + oc * 8 + e] = q2[e];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // not vmcnt: the Y stores stay in flight
    raw_barrier();
    if (tid < 2 * kStemK) {
      const int which = tid / kStemK, col = tid - which * kStemK;
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) a += red[(w * 2 + which) * kStemK + col];
      stats[((long)tm * 2 + which) * kStemK + col] = a;
    }
  }
}
}  // namespace

// Host launcher.  Caller guarantees: Kout % 8 == 0, Kpad % BK == 0 (filter rows zero-padded),
// 16-B aligned tensors, taps.n <= DTF_MAX_TAPS.
// Rows of the BN-statistics slab a forward launch writes (= its M tiles), for the caller's
// workspace sizing; must mirror the tile choice in dtf_conv_igemm.
// -1: automatic, 0: never the DMA kernel, 1: whenever legal (benchmarks / tests)
static int g_conv_dma_mode = -1;
void dtf_conv_set_small_k(int mode) { g_small_k = mode; }
void dtf_conv_set_dma_mode(int mode) { g_conv_dma_mode = mode; }

// The 8-wave DMA kernel needs C % 64 == 0 (one tap per K-step) and 128-wide output tiles.
// Measured (tools/conv_bench.py, batch 256, forced on vs off): it wins only on multi-tap convs
// with C >= 256 (the 3x3 convs of stages 2-3: 1.05-1.11x); on 1x1 convs and C = 128 3x3 convs
// the 2-blocks-per-CU register-staged kernel is 5-28 % faster, so auto mode picks it there.
static bool use_dma_kernel(long M, int Kout, int C, int taps, int bk) {
  if (g_conv_dma_mode == 0 || bk != 64 || C % 64 != 0 || Kout % 128 != 0) return false;
  if (g_conv_dma_mode == 1) return true;
  (void)M;
  return taps > 1 && C >= 256;
}

// halo kernel families (bit 0: 56 x 56 x 64 -> 64k, bit 1: 28 x 28 x 128 -> 128k): 3x3 stride-1
// "same" convs (forward and data gradient)
static int g_halo = 3;
void dtf_conv_set_halo(int on) { g_halo = on; }
// 0: not eligible; 1: the 56 x 56 x 64 family; 2: the 28 x 28 x 128 family
static int halo_family(const ConvGeom& g, const TapTable& taps) {
  if (!g_halo || g.H % kHaloTH || taps.n != 9 || g.sh != 1 || g.sw != 1 || g.P != g.H ||
      g.Q != g.W || g.Ho != g.H || g.Wo != g.W || g.osh != 1 || g.osw != 1 || g.oh0 || g.ow0 ||
      g.acc || g.Kpad != 9 * g.C)
    return 0;
  for (int t = 0; t < 9; ++t)
    if (taps.dh[t] < -1 || taps.dh[t] > 1 || taps.dw[t] < -1 || taps.dw[t] > 1) return 0;
  if (g.C == 64 && g.W == 56 && g.Kout % 64 == 0) return 1;
  if ((g_halo & 2) && g.C == 128 && g.W == 28 && g.Kout % 128 == 0) return 2;
  return 0;
}
static bool use_halo(const ConvGeom& g, const TapTable& taps) { return halo_family(g, taps) != 0; }
// strips per halo block, per family (bit 0: 56 x 56 x 64, bit 1: 28 x 28 x 128)
static int g_halo_st = 0;   // measured: no faster (one 8-wave block per CU), see r2_halo_strips_ab_b2048.txt
void dtf_conv_set_halo_strips(int v) { g_halo_st = v; }
// filter streamed into registers instead of an LDS ring, per family (bit 0: 56 x 56 x 64,
// bit 1: 28 x 28 x 128); see conv3x3_halo_kernel FREG
static int g_halo_freg = 0;
void dtf_conv_set_halo_freg(int v) { g_halo_freg = v; }
// filter-ring depth per halo family: nibble f - 1 of g_halo_stages (0 or 2: the double buffer;
// 3 / 4: deeper rings; family 1 keeps two blocks per CU at 4, family 2 only with two strips)
static int g_halo_stages = 0;
void dtf_conv_set_halo_stages(int v) { g_halo_stages = v; }
// timing probe: the BN-on-load forward without its y stores (wrong results downstream).  Only in
// a probe build (-DDTF_PROBES, tools only): the default build has no such kernel and refuses
#ifdef DTF_PROBES
static int g_bnl_probe = 0;
void dtf_conv_set_bnl_probe(int v) { g_bnl_probe = v; }
#else
static constexpr int g_bnl_probe = 0;
void dtf_conv_set_bnl_probe(int v) {
  if (v) throw std::runtime_error("conv_set_bnl_probe: a timing probe with wrong results; build "
                                  "with DTF_HIP_EXTRA_FLAGS=-DDTF_PROBES (tools only)");
}
#endif

template <int C, int W, int WMW, int NT, int ST, bool BNB, int NSTG>
static void launch_halo_ring(const bf16_t* X, const bf16_t* Wt, bf16_t* Y, const ConvGeom& g,
                             const TapTable& taps, float* stats, const BnBwdEpi& bnb, int tiles,
                             size_t lds, hipStream_t st) {
  auto kern = conv3x3_halo_kernel<C, W, WMW, NT, ST, false, BNB, NSTG>;
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024));
    attr = true;
  }
  if (lds > 160 * 1024) throw std::runtime_error("halo conv: filter ring exceeds LDS");
  hipLaunchKernelGGL(kern, dim3((unsigned)((tiles + ST - 1) / ST), g.Kout / NT),
                     dim3(kThreads * ST), lds, st, X, Wt, Y, g, taps, stats, bnb);
}

template <int C, int W, int WMW, int NT>
static void launch_halo(const bf16_t* X, const bf16_t* Wt, bf16_t* Y, const ConvGeom& g,
                        const TapTable& taps, float* stats, const BnBwdEpi& bnb, int tiles,
                        int strips, hipStream_t st) {
  using Hc = HaloCfg<C, W, WMW, NT>;
  const int nstg = (g_halo_stages >> (C == 64 ? 0 : 4)) & 15;
  const bool freg_on = (g_halo_freg & (C == 64 ? 1 : 2)) != 0;
  if (g.ly) {
    if (bnb.part || freg_on || nstg == 3 || nstg == 4 || strips != 1)
      throw std::runtime_error("halo conv: BN on load needs the default forward ring kernel");
#ifdef DTF_PROBES
    auto kern = g_bnl_probe ? conv3x3_halo_kernel<C, W, WMW, NT, 1, false, false, 2, true, 1>
                            : conv3x3_halo_kernel<C, W, WMW, NT, 1, false, false, 2, true>;
#else
    auto kern = conv3x3_halo_kernel<C, W, WMW, NT, 1, false, false, 2, true>;
#endif
    const size_t lds = Hc::lds(1) + (size_t)2 * C * sizeof(float);    // + the BN scale / shift
    static bool attr[2] = {false, false};
    if (!attr[g_bnl_probe ? 1 : 0]) {
      HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
      attr[g_bnl_probe ? 1 : 0] = true;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)tiles, g.Kout / NT), dim3(kThreads), lds, st,
                       X, Wt, Y, g, taps, stats, bnb);
    return;
  }
  if (!freg_on && (nstg == 3 || nstg == 4)) {
    if (bnb.part) {
      constexpr size_t scratch =
          (size_t)Hc::M * Hc::LDC * 2 + (size_t)(kThreads / (NT / 8)) * 2 * NT * 4;
      const size_t base = Hc::lds(1, nstg);
      const size_t lds = base > scratch ? base : scratch;
      if (nstg == 3) launch_halo_ring<C, W, WMW, NT, 1, true, 3>(X, Wt, Y, g, taps, stats, bnb, tiles, lds, st);
      else launch_halo_ring<C, W, WMW, NT, 1, true, 4>(X, Wt, Y, g, taps, stats, bnb, tiles, lds, st);
    } else if (strips == 2) {
      if (nstg == 3) launch_halo_ring<C, W, WMW, NT, 2, false, 3>(X, Wt, Y, g, taps, stats, bnb, tiles, Hc::lds(2, 3), st);
      else launch_halo_ring<C, W, WMW, NT, 2, false, 4>(X, Wt, Y, g, taps, stats, bnb, tiles, Hc::lds(2, 4), st);
    } else {
      if (nstg == 3) launch_halo_ring<C, W, WMW, NT, 1, false, 3>(X, Wt, Y, g, taps, stats, bnb, tiles, Hc::lds(1, 3), st);
      else launch_halo_ring<C, W, WMW, NT, 1, false, 4>(X, Wt, Y, g, taps, stats, bnb, tiles, Hc::lds(1, 4), st);
    }
    return;
  }
  if (bnb.part) {
    // one strip per block; the BN-backward reduction scratch [OROWS][2][NT] fp32 sits past the
    // staged tile (in the dead filter ring, or past the patch with FREG)
    constexpr size_t scratch = (size_t)Hc::M * Hc::LDC * 2 + (size_t)(kThreads / (NT / 8)) * 2 * NT * 4;
    const bool freg = (g_halo_freg & (C == 64 ? 1 : 2)) != 0;
    const size_t base = freg ? Hc::LDS_FREG : Hc::lds(1);
    const size_t lds = base > scratch ? base : scratch;
    if (freg)
      hipLaunchKernelGGL((conv3x3_halo_kernel<C, W, WMW, NT, 1, true, true>),
                         dim3((unsigned)tiles, g.Kout / NT), dim3(kThreads), lds, st, X, Wt, Y, g,
                         taps, stats, bnb);
    else
      hipLaunchKernelGGL((conv3x3_halo_kernel<C, W, WMW, NT, 1, false, true>),
                         dim3((unsigned)tiles, g.Kout / NT), dim3(kThreads), lds, st, X, Wt, Y, g,
                         taps, stats, bnb);
    return;
  }
  if (strips == 2) {
    static bool attr = false;
    if (!attr) {
      HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_halo_kernel<C, W, WMW, NT, 2>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)Hc::lds(2)));
      attr = true;
    }
    hipLaunchKernelGGL((conv3x3_halo_kernel<C, W, WMW, NT, 2>),
                       dim3((unsigned)((tiles + 1) / 2), g.Kout / NT), dim3(2 * kThreads), Hc::lds(2),
                       st, X, Wt, Y, g, taps, stats, bnb);
  } else if (g_halo_freg & (C == 64 ? 1 : 2)) {
    hipLaunchKernelGGL((conv3x3_halo_kernel<C, W, WMW, NT, 1, true>),
                       dim3((unsigned)tiles, g.Kout / NT), dim3(kThreads), Hc::LDS_FREG, st, X, Wt,
                       Y, g, taps, stats, bnb);
  } else {
    hipLaunchKernelGGL((conv3x3_halo_kernel<C, W, WMW, NT, 1>), dim3((unsigned)tiles, g.Kout / NT),
                       dim3(kThreads), Hc::lds(1), st, X, Wt, Y, g, taps, stats, bnb);
  }
}

// the space-to-depth ResNet stem (4x4 taps over 16 channels -> 64, output 112 x 112)
static int g_stem_halo = 1;
void dtf_conv_set_stem_halo(int v) { g_stem_halo = v; }
static bool use_stem_halo(const ConvGeom& g, const TapTable& taps) {
  if (!g_stem_halo || g.C != kStemC || g.Kout != kStemK || g.Kpad != kStemKD || taps.n != 16 ||
      g.sh != 1 || g.sw != 1 || g.Q != 112 || g.P % kStemTH || g.H != g.P + 3 || g.W != g.Q + 3 ||
      g.Ho != g.P || g.Wo != g.Q || g.osh != 1 || g.osw != 1 || g.oh0 || g.ow0 || g.acc ||
      g.bias || g.relu)
    return false;
  for (int t = 0; t < 16; ++t)
    if (taps.dh[t] != t / 4 || taps.dw[t] != t % 4) return false;
  return true;
}

// the halo kernels also take the fused-BN-backward (BNB) data gradients (A/B knob)
static int g_halo_bnb = 1;
void dtf_conv_set_halo_bnb(int v) { g_halo_bnb = v; }

// M tiles of a launch WITHOUT the halo kernel; W is accepted for API symmetry and ignored
int dtf_conv_stats_rows(long M, int Kout, int C, int taps, int W) {
  (void)W;
  const int BM = use_dma_kernel(M, Kout, C, taps, 64) ? kDmaBM : (Kout <= 64 ? 256 : 128);
  return (int)((M + BM - 1) / BM);
}

// multi-tap convs with C % 64 == 0 and Kout >= 256 whose outputs map one-to-one onto the M rows
// (forward convs, stride-1 data gradients) run as implicit GEMMs on gemm.hip's ping-pong
// kernel (256 x 256 tiles, 1.2-1.3 PF on long-K GEMMs vs ~0.9 for the 256 x 128 DMA kernel)
static int g_conv_gemm = 1;
void dtf_conv_set_gemm(int v) { g_conv_gemm = v; }
int dtf_gemm_conv_part_images(int N, int H, int W, int C, int P, int Q);
static bool use_conv_gemm(const ConvGeom& g, const TapTable& taps) {
  const bool unit = g.osh == 1 && g.osw == 1 && g.oh0 == 0 && g.ow0 == 0 && g.Ho == g.P &&
                    g.Wo == g.Q;
  // strided-dgrad phase classes qualify too (any tap count, no masked-residual epilogue)
  // bit 1: also 64 < Kout <= 128 on the 256 x 128 ping-pong tile -- measured SLOWER than the
  // halo / register kernels (profiles/measurements/r2_conv_kout128_pingpong_ab.txt), off
  const bool wide = g.Kout >= 256 || ((g_conv_gemm & 2) && g.Kout > 64 && g.Kout <= 128);
  // strided 1x1 forward (the projection shortcuts, 1 tap): on the persistent GEMM when its whole
  // input fits one buffer descriptor (gemm.hip launch_gemm_pp2); the register kernel ran these
  // at 2.5 TB/s / 0.42 PF (s1b0proj 977 us, s2b0proj 666 us at b1984, profiles/r6)
  // (an input past one descriptor runs as batch parts, dtf_gemm_conv_part_images)
  const bool proj = taps.n == 1 && (g.sh > 1 || g.sw > 1) && g.C >= 128 && g.Kout > 128 &&
                    !g.acc && dtf_gemm_conv_part_images(g.N, g.H, g.W, g.C, g.P, g.Q) >= 0 &&
                    g.N < 2048 && g.H < 1000 && g.W < 1000;
  return (g_conv_gemm & 1) && g.C % 64 == 0 && wide && g.Kout % 8 == 0 && taps.n <= 9 &&
         (unit ? (taps.n > 1 || proj) : g.acc != 2) && g.Kpad == taps.n * g.C && !g.bias &&
         !g.relu && g.H < 16384 && g.W < 32768;
}
void dtf_gemm_conv(const bf16_t* X, const bf16_t* Wt, bf16_t* Y, int N, int H, int W, int C,
                   int P, int Q, int sh, int sw, int Kout, int ntaps, const int* dh, const int* dw,
                   int Ho, int Wo, int osh, int osw, int oh0, int ow0,
                   float* stats, const bf16_t* Cin, const bf16_t* acc_src,
                   const uint8_t* acc_mask, hipStream_t st);

// M tiles (= BN-statistics slab rows) of exactly the kernel dtf_conv_igemm will pick for this
// forward launch (no fused BN-backward epilogue)
int dtf_conv_tile_rows(const ConvGeom& g, const TapTable& taps, int bnb) {
  if (bnb) {   // a fused-BN-backward data gradient (the dispatch of dtf_conv_igemm with bnb.part)
    if (g.C % 32 == 0 && !g.bias && !g.relu && use_halo(g, taps) && g_halo_bnb)
      return g.N * (g.H / kHaloTH);
    return dtf_conv_stats_rows((long)g.N * g.P * g.Q, g.Kout, g.C, taps.n, 0);
  }
  if (use_conv_gemm(g, taps)) return (int)(((long)g.N * g.P * g.Q + 255) / 256);
  if (g.C % 32 == 0 && use_halo(g, taps)) return g.N * (g.H / kHaloTH);
  if (use_stem_halo(g, taps)) return g.N * (g.P / kStemTH);
  const long M = (long)g.N * g.P * g.Q;
  return dtf_conv_stats_rows(M, g.Kout, g.C, taps.n, 0);
}

static int g_conv_nt = 0;   // measured neutral on ResNet-50 b2048 (DTF_STORE_NT A/B)
void dtf_conv_set_nt(int v) { g_conv_nt = v; }

// the forward conv can take its input through a BatchNorm + ReLU on load (halo kernels, the
// default forward ring configuration of the family)
bool dtf_conv_bnl_ok(const ConvGeom& g, const TapTable& taps) {
  const int fam = halo_family(g, taps);
  if (!fam || (g_halo_freg & fam) || (g_halo_st & fam)) return false;
  const int nstg = (g_halo_stages >> (fam == 1 ? 0 : 4)) & 15;
  return nstg != 3 && nstg != 4;
}

void dtf_conv_igemm(const bf16_t* X, const bf16_t* Wt, bf16_t* Y, const ConvGeom& g_in,
                    const TapTable& taps, int bk, float* stats, const BnBwdEpi& bnb,
                    hipStream_t st) {
  ConvGeom g = g_in;
  g.nt = g_conv_nt;
  if (bnb.part && (stats || !bnb.x || !bnb.mean || !bnb.invstd ||
                   (bnb.mkind == 1 && !bnb.mask) || (bnb.mkind == 2 && !(bnb.fsc && bnb.fsh))))
    throw std::runtime_error("conv: bad fused BN-backward epilogue arguments");
  if (taps.n <= 0 || taps.n > DTF_MAX_TAPS) throw std::runtime_error("conv: bad tap count");
  if (g.Kout % 8) throw std::runtime_error("conv: Kout % 8 != 0");
  // buffer descriptors are rebased per tile at its first image: only a few images (and the
  // filter) must fit 32-bit offsets; the row count itself is a 32-bit int
  const double ibytes = 2.0 * g.H * g.W * g.C, wbytes = 2.0 * g.Kout * g.Kpad;
  const double m = (double)g.N * g.P * g.Q;
  const double span = (double)(255 / (g.P * g.Q) + 2);   // images one 256-row tile touches
  if (ibytes * span >= 2147483647.0 || wbytes >= 2147483647.0 || m >= 2147483647.0 ||
      (double)g.N * g.Ho * g.Wo >= 2147483647.0)
    throw std::runtime_error("conv: image / filter too large for 32-bit buffer offsets");
  const bool narrow = g.Kout <= 64;        // 256 x 64 tile for 64-wide layers
  const bool epi = g.bias || g.relu;       // fused bias / ReLU: register kernel only
  if (epi && (bnb.part || g.acc))
    throw std::runtime_error("conv: fused bias/ReLU epilogue excludes BN / accumulate epilogues");
  if (g.ly) {                              // BN + ReLU on load: the halo forward kernel only
    if (!dtf_conv_bnl_ok(g, taps) || !g.lsc || !g.lsh || bnb.part || epi)
      throw std::runtime_error("conv: BN on load needs a halo-family forward conv");
    const int tiles = g.N * (g.H / kHaloTH);
    if (halo_family(g, taps) == 1)
      launch_halo<64, 56, 2, 64>(X, Wt, Y, g, taps, stats, bnb, tiles, 1, st);
    else
      launch_halo<128, 28, 1, 128>(X, Wt, Y, g, taps, stats, bnb, tiles, 1, st);
    return;
  }
  if (!bnb.part && use_stem_halo(g, taps)) {
    using Sc = StemCfg<112>;
    static bool attr = false;
    if (!attr) {
      HIP_CHECK(hipFuncSetAttribute((const void*)conv_stem_halo_kernel<112>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)Sc::LDS));
      attr = true;
    }
    hipLaunchKernelGGL(conv_stem_halo_kernel<112>, dim3((unsigned)(g.N * (g.P / kStemTH))),
                       dim3(kThreads), Sc::LDS, st, X, Wt, Y, g, stats);
    return;
  }
  if (g.C % 32 != 0) {
    if (g.Kpad % 32) throw std::runtime_error("conv: Kpad % 32 != 0");
    if (g.C % 8 == 0) {                    // chunk gather (stem / MNIST conv1, C padded to 8)
      if (narrow) launch_cfg<4, 1, 32, 2>(X, Wt, Y, g, taps, stats, bnb, st);
      else launch_cfg<2, 2, 32, 2>(X, Wt, Y, g, taps, stats, bnb, st);
    } else {
      if (narrow) launch_cfg<4, 1, 32, 1>(X, Wt, Y, g, taps, stats, bnb, st);
      else launch_cfg<2, 2, 32, 1>(X, Wt, Y, g, taps, stats, bnb, st);
    }
    return;
  }
  if (!bnb.part && use_conv_gemm(g, taps)) {
    dtf_gemm_conv(X, Wt, Y, g.N, g.H, g.W, g.C, g.P, g.Q, g.sh, g.sw, g.Kout, taps.n, taps.dh,
                  taps.dw, g.Ho, g.Wo, g.osh, g.osw, g.oh0, g.ow0, stats,
                  g.acc == 1 ? Y : nullptr, g.acc == 2 ? g.acc_src : nullptr,
                  g.acc == 2 ? g.acc_mask : nullptr, st);
    return;
  }
  if (!epi && use_halo(g, taps) && (!bnb.part || (g_halo_bnb && !stats))) {
    const int fam = halo_family(g, taps);
    const int tiles = g.N * (g.H / kHaloTH);
    if (fam == 1)
      launch_halo<64, 56, 2, 64>(X, Wt, Y, g, taps, stats, bnb, tiles, (g_halo_st & 1) ? 2 : 1, st);
    else
      launch_halo<128, 28, 1, 128>(X, Wt, Y, g, taps, stats, bnb, tiles, (g_halo_st & 2) ? 2 : 1, st);
    return;
  }
  if (!epi && use_dma_kernel((long)m, g.Kout, g.C, taps.n, bk) && g.Kpad % 64 == 0) {
    const long tiles = (((long)m + kDmaBM - 1) / kDmaBM) * (g.Kout / kDmaBN);
    if (bnb.part)
      hipLaunchKernelGGL(conv_igemm_dma_kernel<true>, dim3((unsigned)tiles), dim3(kDmaThreads), 0,
                         st, X, Wt, Y, g, taps, stats, bnb);
    else
      hipLaunchKernelGGL(conv_igemm_dma_kernel<false>, dim3((unsigned)tiles), dim3(kDmaThreads), 0,
                         st, X, Wt, Y, g, taps, stats, bnb);
    return;
  }
  // small-K 1x1 convs (one or two 64-deep K-steps: latency-bound blocks): optionally BK 32 with
  // 16-KB stages -> more blocks per CU (g_small_k bit 1; A/B-measured by tools/conv_bench.py)
  if ((g_small_k & 2) && taps.n == 1 && g.C <= 128) bk = 32;
  if ((g_small_k & 4) && taps.n == 1) bk = 32;            // every 1x1 conv
  if ((g_small_k & 8) && !use_dma_kernel((long)m, g.Kout, g.C, taps.n, 64)) bk = 32;   // all reg.
  if (bk == 64 && g.C % 64 == 0) {
    if (narrow) launch_cfg<4, 1, 64, 0>(X, Wt, Y, g, taps, stats, bnb, st);
    else launch_cfg<2, 2, 64, 0>(X, Wt, Y, g, taps, stats, bnb, st);
  } else {
    if (narrow) launch_cfg<4, 1, 32, 0>(X, Wt, Y, g, taps, stats, bnb, st);
    else launch_cfg<2, 2, 32, 0>(X, Wt, Y, g, taps, stats, bnb, st);
  }
}

// The phase classes of a strided data gradient in one launch (conv_igemm_grouped_kernel).  g0:
// the shared geometry (oh0 / ow0 / Kpad are per class); dh / dw: each class's taps.  Returns
// false -- nothing launched -- when the classes would not all take the BK-32 register kernel
// dtf_conv_igemm picks for them, or do not have equal tile grids; the caller then launches them
// one by one.
bool dtf_conv_igemm_grouped(const bf16_t* X, bf16_t* Y, const ConvGeom& g0, int ncls,
                            const bf16_t* const* wts, const int* oh0, const int* ow0,
                            const int* kpad, const std::vector<std::vector<int>>& dh,
                            const std::vector<std::vector<int>>& dw, const BnBwdEpi& bnb,
                            const int* row0, hipStream_t st) {
  if (ncls < 2 || ncls > kGrpMax || g0.C % 32 || g0.bias || g0.relu || g0.ly || g0.acc == 2 ||
      !(g_small_k & 8) || g0.Kout % 8)
    return false;
  // not with the fused BN-backward sums: grouped, that epilogue ran 1.97 vs 1.78 ms split
  // (56x56x128 stride 2, b1984; tools/conv_gap.py)
  if (bnb.part) return false;
  ConvGroup grp{};
  grp.n = ncls;
  ConvGeom g = g0;
  g.nt = g_conv_nt;
  const long m = (long)g.N * g.P * g.Q;
  int max_nk = 0;
  for (int c = 0; c < ncls; ++c) {
    const int nt = (int)dh[c].size();
    if (nt < 1 || nt > kGrpTaps || (int)dw[c].size() != nt || kpad[c] % 32 ||
        kpad[c] < nt * g.C)
      return false;
    TapTable t{};
    t.n = nt;
    grp.taps[c].n = nt;
    for (int i = 0; i < nt; ++i) {
      t.dh[i] = grp.taps[c].dh[i] = dh[c][i];
      t.dw[i] = grp.taps[c].dw[i] = dw[c][i];
    }
    ConvGeom gc = g;
    gc.oh0 = oh0[c];
    gc.ow0 = ow0[c];
    gc.Kpad = kpad[c];
    // the kernel dtf_conv_igemm would choose must be the register kernel
    if (use_conv_gemm(gc, t) || use_halo(gc, t) ||
        (use_dma_kernel(m, gc.Kout, gc.C, nt, 64) && gc.Kpad % 64 == 0))
      return false;
    const double wbytes = 2.0 * gc.Kout * gc.Kpad;
    if (wbytes >= 2147483647.0) return false;
    grp.Wt[c] = wts[c];
    grp.g[c] = gc;
    grp.bnb[c] = bnb;
    grp.bnb[c].row0 = row0 ? row0[c] : 0;
    max_nk = std::max(max_nk, (nt * g.C + 31) / 32);
  }
  const double ibytes = 2.0 * g.H * g.W * g.C;
  const double span = (double)(255 / (g.P * g.Q) + 2);
  if (ibytes * span >= 2147483647.0 || m >= 2147483647.0 ||
      (double)g.N * g.Ho * g.Wo >= 2147483647.0)
    return false;
  const bool narrow = g.Kout <= 64;
  const int BM = narrow ? 256 : 128, BN = narrow ? 64 : 128;
  const long tiles = ((m + BM - 1) / BM) * ((g.Kout + BN - 1) / BN) * ncls;
  if (tiles >= (1L << 31)) return false;
  const size_t stage = (size_t)(BM + BN) * 32 * sizeof(bf16_t) *
                           ((max_nk > 1 || !(g_small_k & 1)) ? 2 : 1) +
                       2 * DTF_MAX_TAPS * sizeof(int);
  const int OROWS = kThreads / (BN / 8);
  const size_t scratch = bnb.part ? (size_t)OROWS * 2 * BN : (size_t)2 * kThreads;
  const size_t epi = (size_t)BM * (BN + 8) * sizeof(bf16_t) + scratch * sizeof(float);
  const size_t lds = stage > epi ? stage : epi;
  const dim3 grid((unsigned)tiles), blk(kThreads);
  const bool hi = !bnb.part && (g_small_k & 16);
  if (narrow) {
    if (hi) hipLaunchKernelGGL((conv_igemm_grouped_kernel<4, 1, false, true>), grid, blk, lds, st, X, Y, grp);
    else hipLaunchKernelGGL((conv_igemm_grouped_kernel<4, 1, false, false>), grid, blk, lds, st, X, Y, grp);
  } else {
    if (hi) hipLaunchKernelGGL((conv_igemm_grouped_kernel<2, 2, false, true>), grid, blk, lds, st, X, Y, grp);
    else hipLaunchKernelGGL((conv_igemm_grouped_kernel<2, 2, false, false>), grid, blk, lds, st, X, Y, grp);
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// Batched filter transpose for the data gradient: every conv's bf16 filter [K][T][C] -> [C][T][K]
// (the dgrad GEMM's B operand) in ONE launch per step instead of one torch copy kernel per conv
// (53 launches / ResNet-50 step).  Block = one 64 x 64 (k, c) tile of one tap of one filter,
// staged through a padded LDS tile so both the reads (along c) and the writes (along k) are
// coalesced.  Jobs are found by a scan of the (<= kWtMaxJobs) cumulative tile counts.
constexpr int kWtMaxJobs = 48;
struct WtJobs {
  const bf16_t* src[kWtMaxJobs];
  bf16_t* dst[kWtMaxJobs];
  int K[kWtMaxJobs], T[kWtMaxJobs], C[kWtMaxJobs];
  int tile_end[kWtMaxJobs];     // exclusive prefix sum of T * ceil(K/64) * ceil(C/64)
  int n;
};

namespace {
__global__ void __launch_bounds__(256) filter_transpose_kernel(const WtJobs jobs) {
  __shared__ bf16_t tile[64][66];
  const int b = blockIdx.x;
  int j = 0;
  while (j < jobs.n - 1 && b >= jobs.tile_end[j]) ++j;     // wave-uniform scan
  const int start = j ? jobs.tile_end[j - 1] : 0;
  const int K = jobs.K[j], T = jobs.T[j], C = jobs.C[j];
  const int tk = (K + 63) / 64, tc = (C + 63) / 64;
  const int local = b - start;
  const int t = local / (tk * tc);
  const int rem = local % (tk * tc);
  const int k0 = (rem / tc) * 64, c0 = (rem % tc) * 64;
  const bf16_t* src = jobs.src[j];
  bf16_t* dst = jobs.dst[j];
  const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;   // 64 columns x 4 rows per pass
#pragma unroll 4
  for (int r = ly; r < 64; r += 4) {
    const int k = k0 + r, c = c0 + lx;
    tile[r][lx] = (k < K && c < C) ? src[((long)k * T + t) * C + c] : (bf16_t)0;
  }
  __syncthreads();
#pragma unroll 4
  for (int r = ly; r < 64; r += 4) {
    const int c = c0 + r, k = k0 + lx;
    if (c < C && k < K) dst[((long)c * T + t) * K + k] = tile[lx][r];
  }
}
}  // namespace

void dtf_filter_transpose(const WtJobs& jobs, hipStream_t st) {
  if (jobs.n <= 0) return;
  if (jobs.n > kWtMaxJobs) throw std::runtime_error("filter_transpose: too many jobs");
  hipLaunchKernelGGL(filter_transpose_kernel, dim3((unsigned)jobs.tile_end[jobs.n - 1]), dim3(256),
                     0, st, jobs);
}
