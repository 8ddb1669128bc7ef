// Weight-gradient implicit GEMM on MFMA (SURVEY.md K3b/K5b/N-K1 wgrad), NHWC bf16 in, fp32 out.
//
//   dW[k, t*C + c] = sum_m dY[m, k] * X[n(m), p(m)*sh + dh_t, q(m)*sw + dw_t, c]
//
// GEMM rows = Kout, cols = T*C, reduction over the M = N*P*Q output pixels (huge: split-K).
// Both operands are contiguous in their GEMM row/col index and strided in the reduction index,
// so tiles are staged in LDS pixel-major ([m][channels], straight 16-B global loads) and the MFMA
// fragments (8 consecutive reduction indices per lane) are read with the gfx950 hardware
// transpose read ds_read_b64_tr_b16 (cdna_hip_programming.md §5.5 T10): two 8-byte transposed
// reads per 16x16x32 fragment.
// Split-K partial tiles are combined with fp32 atomic adds into a zeroed dW (Guideline 12:
// few splits per tile, each tile's adds are 16 contiguous floats per 16-lane group).
#include <stdexcept>
#include <string>

#include "common.h"

#define DTF_MAX_TAPS 64

struct TapTableW {
  int n;
  int dh[DTF_MAX_TAPS];
  int dw[DTF_MAX_TAPS];
};

struct WgradGeom {
  int N, H, W, C;   // input X
  int P, Q;         // dY spatial
  int sh, sw;
  int Kout;
  int ldw;          // dW row stride (>= T*C)
  long m_per_split; // reduction pixels per split (multiple of BKM)
};

namespace {
constexpr int kThreads = 256;
constexpr int BM = 128, BN = 128, BKM = 64;
constexpr int LDA = BM + 16;   // padded LDS row (elements): 288 B rows = 8-bank shift per row
constexpr int LDB = BN + 16;
// rows r and r+8 are read by the two 16-lane groups of one 32-lane half of a transposed read:
// shift rows with bit 3 set by 128 B (32 banks) so the half's 8 rows cover all 64 banks.
DTF_DEV int roff(int r, int ld) { return r * ld + ((r >> 3) & 1) * 64; }
constexpr int OPER_A = BKM * LDA + 64;
constexpr int OPER_B = BKM * LDB + 64;

typedef __attribute__((ext_vector_type(4))) short s4_t;
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

DTF_DEV s4_t tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(p));
}

template <bool GENERIC>
__global__ void __launch_bounds__(kThreads, 2)
conv_wgrad_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                  float* __restrict__ dW, const WgradGeom g, const TapTableW taps) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  constexpr int STAGE = OPER_A + OPER_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int TC = taps.n * g.C;
  const int tiles_m = (g.Kout + BM - 1) / BM;
  const int tiles_n = (TC + BN - 1) / BN;
  const int tile = blockIdx.x % (tiles_m * tiles_n);
  const int split = blockIdx.x / (tiles_m * tiles_n);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int k0 = tm * BM, j0 = tn * BN;
  const long M = (long)g.N * g.P * g.Q;
  const long ms = (long)split * g.m_per_split;
  long me = ms + g.m_per_split;
  if (me > M) me = M;
  const int nk = (int)((me - ms + BKM - 1) / BKM);

  // thread -> (row, chunk) for staging: 16 chunks of 8 channels per 128-wide row
  const int cc = tid & 15;
  const int rr = tid >> 4;         // 0..15, rows rr + 16*i
  uint4 ra[4], rb[4];

  // per-chunk tap / channel for the B (X) gather (fixed across K-steps)
  const int jc = j0 + cc * 8;
  int bt = 0, bc = 0;
  if (!GENERIC && jc < TC) { bt = jc / g.C; bc = jc - bt * g.C; }
  const int bdh = (!GENERIC && jc < TC) ? taps.dh[bt] : 0;
  const int bdw = (!GENERIC && jc < TC) ? taps.dw[bt] : 0;
  const bool a_col_ok = (k0 + cc * 8) < g.Kout;

  auto load_stage = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long m = ms + (long)kt * BKM + rr + 16 * i;
      const bool mok = m < me;
      // A: dY row m, channels k0 + cc*8
      if (mok && a_col_ok)
        ra[i] = *reinterpret_cast<const uint4*>(dY + m * g.Kout + k0 + cc * 8);
      else
        ra[i] = make_uint4(0, 0, 0, 0);
      const long mm = mok ? m : 0;
      const int q = (int)(mm % g.Q);
      const long t = mm / g.Q;
      const int p = (int)(t % g.P);
      const int n = (int)(t / g.P);
      if constexpr (!GENERIC) {
        const int h = p * g.sh + bdh, w = q * g.sw + bdw;
        if (mok && jc < TC && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W)
          rb[i] = *reinterpret_cast<const uint4*>(X + (((long)n * g.H + h) * g.W + w) * g.C + bc);
        else
          rb[i] = make_uint4(0, 0, 0, 0);
      } else {
        uint32_t wv[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          uint32_t pair = 0;
#pragma unroll
          for (int e1 = 0; e1 < 2; ++e1) {
            const int j = jc + e2 * 2 + e1;
            uint32_t v = 0;
            if (mok && j < TC) {
              const int tt = j / g.C, c = j - tt * g.C;
              const int h = p * g.sh + taps.dh[tt], w = q * g.sw + taps.dw[tt];
              if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W)
                v = X[(((long)n * g.H + h) * g.W + w) * g.C + c];
            }
            pair |= v << (16 * e1);
          }
          wv[e2] = pair;
        }
        rb[i] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
    }
  };
  auto store_stage = [&](int buf) {
    bf16_t* sa = lds + buf * STAGE;
    bf16_t* sb = sa + OPER_A;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<uint4*>(sa + roff(rr + 16 * i, LDA) + cc * 8) = ra[i];
      *reinterpret_cast<uint4*>(sb + roff(rr + 16 * i, LDB) + cc * 8) = rb[i];
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    load_stage(0);
    store_stage(0);
  }
  __syncthreads();
  const int gq = lane >> 4;          // 16-lane group = 8-pixel slice of the 32-deep MFMA k
  const int li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_stage(kt + 1);
    const bf16_t* sa = lds + cur * STAGE;
    const bf16_t* sb = sa + OPER_A;
#pragma unroll
    for (int ks = 0; ks < BKM / 32; ++ks) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r0 = 32 * ks + 8 * gq + tq, c0 = wm * 64 + 16 * i + 4 * tp;
        const s4_t lo = tr_read(sa + roff(r0, LDA) + c0);
        const s4_t hi = tr_read(sa + roff(r0 + 4, LDA) + c0);
        af[i] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r0 = 32 * ks + 8 * gq + tq, c0 = wn * 64 + 16 * j + 4 * tp;
        const s4_t lo = tr_read(sb + roff(r0, LDB) + c0);
        const s4_t hi = tr_read(sb + roff(r0 + 4, LDB) + c0);
        bfr[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_stage(cur ^ 1);
    __syncthreads();
  }
  // epilogue: fp32 atomic add (split-K) — rows = k, cols = j
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = j0 + wn * 64 + 16 * j + li;
      if (col >= TC) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = k0 + wm * 64 + 16 * i + 4 * gq + r;
        if (row < g.Kout) atomicAdd(dW + (long)row * g.ldw + col, acc[i][j][r]);
      }
    }
}
}  // namespace

int dtf_conv_wgrad_splits(long M, int Kout, int TC) {
  const long tiles = (long)((Kout + BM - 1) / BM) * ((TC + BN - 1) / BN);
  long splits = (1024 + tiles - 1) / tiles;              // ~4 blocks per CU in flight
  const long max_splits = (M + 4 * BKM - 1) / (4 * BKM);  // >= 4 K-steps per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  return (int)splits;
}

// dW must be zero-filled by the caller (atomic accumulation).
void dtf_conv_wgrad(const bf16_t* X, const bf16_t* dY, float* dW, WgradGeom g,
                    const TapTableW& taps, hipStream_t st) {
  if (taps.n <= 0 || taps.n > DTF_MAX_TAPS) throw std::runtime_error("wgrad: bad tap count");
  if (g.Kout % 8) throw std::runtime_error("wgrad: Kout % 8 != 0");
  const long M = (long)g.N * g.P * g.Q;
  const int TC = taps.n * g.C;
  const int splits = dtf_conv_wgrad_splits(M, g.Kout, TC);
  long mps = (M + splits - 1) / splits;
  mps = ((mps + BKM - 1) / BKM) * BKM;
  g.m_per_split = mps;
  const int nsplit = (int)((M + mps - 1) / mps);
  const long tiles = (long)((g.Kout + BM - 1) / BM) * ((TC + BN - 1) / BN);
  const size_t lds = (size_t)2 * (OPER_A + OPER_B) * sizeof(bf16_t);
  const bool generic = (g.C % 8) != 0;
  if (generic)
    hipLaunchKernelGGL(conv_wgrad_kernel<true>, dim3((unsigned)(tiles * nsplit)), dim3(kThreads),
                       lds, st, X, dY, dW, g, taps);
  else
    hipLaunchKernelGGL(conv_wgrad_kernel<false>, dim3((unsigned)(tiles * nsplit)), dim3(kThreads),
                       lds, st, X, dY, dW, g, taps);
}
