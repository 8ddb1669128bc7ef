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
  long slab;        // floats per split slab (Kout * ldw)
};

namespace {
constexpr int kThreads = 256;
constexpr int BM = 128, BN = 128, BKM = 64;
constexpr int LDA = BM + 16;   // padded LDS row (elements): 288 B rows = 8-bank shift per row
constexpr int LDB = BN + 16;
// rows r and r+8 are read by the two 16-lane groups of one 32-lane half of a transposed read;
// with a 288-B pitch they land on the same banks, so rows with bit 3 set store their two 128-B
// column halves swapped (a permutation within the row: element (r, c) lives at column
// c ^ 64): the half's 8 rows then cover all 64 banks.
DTF_DEV int lidx(int r, int c, int ld) { return r * ld + (c ^ (((r >> 3) & 1) << 6)); }
constexpr int OPER_A = BKM * LDA;
constexpr int OPER_B = BKM * LDB;

typedef __attribute__((ext_vector_type(4))) short s4_t;
typedef __attribute__((address_space(3))) s4_t lds_s4_t;
constexpr uint32_t kOOB = 0xFFFFFFF0u;   // byte offset the buffer range check always rejects

DTF_DEV __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
DTF_DEV uint4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
DTF_DEV uint32_t bload2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}

DTF_DEV s4_t tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(p));
}

template <bool GENERIC, bool TR>
__global__ void __launch_bounds__(kThreads, 2)
conv_wgrad_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                  float* __restrict__ dW, const WgradGeom g, const TapTableW taps, int mode) {
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
  const int M = g.N * g.P * g.Q;               // host guarantees < 2^31
  const int ms = split * (int)g.m_per_split;
  int me = ms + (int)g.m_per_split;
  if (me > M) me = M;
  const int nk = (me - ms + BKM - 1) / BKM;

  // thread -> (row, chunk) for staging: 16 chunks of 8 channels per 128-wide row
  const int cc = tid & 15;
  const int rr = tid >> 4;         // 0..15, rows rr + 16*i
  uint4 ra[4], rb[4];

  // tap table -> LDS with wave-uniform (scalar) kernel-argument reads only; per-lane lookups
  // then come from LDS (never per-lane vector loads from the kernarg segment)
  int* lds_taps = reinterpret_cast<int*>(lds + 2 * STAGE);   // [2][DTF_MAX_TAPS]
  if (tid == 0)
    for (int t = 0; t < taps.n; ++t) { lds_taps[t] = taps.dh[t]; lds_taps[DTF_MAX_TAPS + t] = taps.dw[t]; }
  __syncthreads();

  // per-chunk tap / channel for the B (X) gather (fixed across K-steps)
  const int jc = j0 + cc * 8;
  const bool b_col_ok = jc < TC;
  const int bt = b_col_ok ? jc / g.C : 0;
  const int bc = jc - bt * g.C;
  const int bdh = lds_taps[bt], bdw = lds_taps[DTF_MAX_TAPS + bt];
  const bool a_col_ok = (k0 + cc * 8) < g.Kout;
  // descriptors rebased at this split's first dY row / first X image (64-bit pointer math):
  // the 32-bit buffer offsets only span one split, never the whole tensor
  const int PQ = g.P * g.Q;
  const int n_lo = ms / PQ, n_hi = max(n_lo, (me - 1) / PQ);
  const long img = (long)g.H * g.W * g.C;
  const auto rx = rsrc(X + n_lo * img, (uint32_t)((n_hi - n_lo + 1) * img * 2));
  const auto ry = rsrc(dY + (long)ms * g.Kout, (uint32_t)max(me - ms, 0) * g.Kout * 2u);
  const int HW = g.H * g.W;

  // branch-free loads: padding / out-of-range lanes get an out-of-range buffer offset -> zeros
  auto load_stage = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = ms + kt * BKM + rr + 16 * i;
      const bool mok = m < me;
      ra[i] = bload16(ry, (mok && a_col_ok) ? (uint32_t)(((m - ms) * g.Kout + k0 + cc * 8) * 2) : kOOB);
      const int mm = mok ? m : ms;
      const int q = mm % g.Q;
      const int t = mm / g.Q;
      const int p = t % g.P;
      const int n = t / g.P - n_lo;
      if constexpr (!GENERIC) {
        const int h = p * g.sh + bdh, w = q * g.sw + bdw;
        const bool ok = mok && b_col_ok && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
        rb[i] = bload16(rx, ok ? (uint32_t)(((n * HW + h * g.W + w) * g.C + bc) * 2) : kOOB);
      } else {
        uint32_t wv[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          uint32_t pair = 0;
#pragma unroll
          for (int e1 = 0; e1 < 2; ++e1) {
            const int j = jc + e2 * 2 + e1;
            const int tt = j < TC ? j / g.C : 0;
            const int c = j - tt * g.C;
            const int h = p * g.sh + lds_taps[tt], w = q * g.sw + lds_taps[DTF_MAX_TAPS + tt];
            const bool ok = mok && j < TC && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
            pair |= bload2(rx, ok ? (uint32_t)(((n * HW + h * g.W + w) * g.C + c) * 2) : kOOB)
                    << (16 * e1);
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
      *reinterpret_cast<uint4*>(sa + lidx(rr + 16 * i, cc * 8, LDA)) = ra[i];
      *reinterpret_cast<uint4*>(sb + lidx(rr + 16 * i, cc * 8, LDB)) = rb[i];
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
    const int cur = mode == 2 ? 0 : (kt & 1);
    if (kt + 1 < nk) load_stage(kt + 1);
    const bf16_t* sa = lds + cur * STAGE;
    const bf16_t* sb = sa + OPER_A;
#pragma unroll
    for (int ks = 0; ks < BKM / 32; ++ks) {
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (TR) {
          const int r0 = 32 * ks + 8 * gq + tq, c0 = wm * 64 + 16 * i + 4 * tp;
          const s4_t lo = tr_read(sa + lidx(r0, c0, LDA));
          const s4_t hi = tr_read(sa + lidx(r0 + 4, c0, LDA));
          af[i] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        } else {
          const int c = wm * 64 + 16 * i + li;
#pragma unroll
          for (int e = 0; e < 8; ++e) af[i][e] = (short)sa[lidx(32 * ks + 8 * gq + e, c, LDA)];
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (TR) {
          const int r0 = 32 * ks + 8 * gq + tq, c0 = wn * 64 + 16 * j + 4 * tp;
          const s4_t lo = tr_read(sb + lidx(r0, c0, LDB));
          const s4_t hi = tr_read(sb + lidx(r0 + 4, c0, LDB));
          bfr[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        } else {
          const int c = wn * 64 + 16 * j + li;
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[j][e] = (short)sb[lidx(32 * ks + 8 * gq + e, c, LDB)];
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (mode >= 1) __syncthreads();
    if (kt + 1 < nk) store_stage(mode == 2 ? 0 : (cur ^ 1));
    __syncthreads();
  }
  // epilogue: this split's fp32 partial tile goes into its own slab (split s writes
  // dW + s * slab); a separate launch sums the slabs in split order -> deterministic, no atomics.
  // The accumulators are staged through LDS by VALU moves (never consumed directly as memory-op
  // data right behind the MFMA chain) after explicit wait states, then stored row-coalesced.
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  constexpr int LDO = BN + 4;                       // fp32 tile [BM][BN+4] = 66 KB
  float* so = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[i][j][r] + 0.0f;
        so[(wm * 64 + 16 * i + 4 * gq + r) * LDO + wn * 64 + 16 * j + li] = v;
      }
  __syncthreads();
  float* out = dW + (long)split * g.slab;
  for (int idx = tid; idx < BM * BN; idx += kThreads) {
    const int r = idx / BN, c = idx % BN;
    const int row = k0 + r, col = j0 + c;
    if (row < g.Kout && col < TC) out[(long)row * g.ldw + col] = so[r * LDO + c];
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA variant (C % 8 == 0, M < 2^24).  The r1 kernel above stages both operands through
// VGPRs + ds_write_b128 into padded rows; at 2 blocks/CU that write pass (≈13 LDS cycles per
// 1-KB wave-instruction) plus the transposed fragment reads exceeded the MFMA time per K-step
// (profiles/r1_conv_roofline: 3x3 wgrad at 0.19-0.20 of the MFMA roof).  Here every 16-B piece
// goes global -> LDS with `buffer_load_dwordx4 ... lds` (no staging VGPRs, ≈4 LDS cycles per
// KB), double-buffered: the DMA of K-step k+1 is issued right after the barrier that publishes
// K-step k, then the MFMAs of k run while it flies (cdna_hip_programming.md §5 "glds, 2 LDS
// buffers, BK=64, vmcnt(0) + plain __syncthreads()").
//
// LDS image: unpadded pixel-major rows ([64 pixels][128 cols] per operand), 16-B chunks
// XOR-swizzled per row so the ds_read_b64_tr_b16 fragment reads are conflict-free: a 32-lane
// half of a transposed read touches rows {0-3, 8-11} (+32ks, +4) at one 32-B column pair, so
// logical chunk c of row r lives in slot c ^ swz(r), swz(r) = 2 * ((r & 3) | ((r >> 3) & 1) << 2)
// -> the 8 rows land on the 8 distinct 32-B bank groups of a 256-B bank row.  The DMA writes
// lane-linearly, so the swizzle is applied on the SOURCE side (lane in slot s fetches chunk
// s ^ swz(r)).  Pixel -> (n, p, q) uses an fp32 reciprocal divmod (exact for m < 2^24).
// Row widths of the two images depend on the wave layout (WM x WN waves of 64 x 64): 128-wide
// tiles (2 x 2, the default) give 256-B rows; the narrow layout for Kout <= 64 (1 x 4: 64 x 256
// tile, no half-empty M tile) gives 128-B dY rows and 512-B X rows.  Conflict-free swizzles for
// the tr-read half {rows 0-3, 8-11} x one 32-B column pair:
//   256 / 512-B rows (bank-row aligned): slot = c ^ 2 * ((r & 3) | ((r >> 3) & 1) << 2)
//   128-B rows (two rows per bank row):  slot = c ^ 2 * (((r >> 1) & 1) | ((r >> 3) & 1) << 1)
template <int ROWB>
DTF_DEV int wswz(int r) {
  if constexpr (ROWB == 128) return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1;
  else return (((r & 3) | (((r >> 3) & 1) << 2)) << 1);
}
template <int W>   // W = row width in elements
DTF_DEV int lds_el(int r, int c) { return r * W + (((c >> 3) ^ wswz<W * 2>(r)) << 3) + (c & 7); }
DTF_DEV void fdivmod(int m, int d, float inv, int& q, int& r) {
  const int t = (int)((float)m * inv);
  const int rem = m - t * d;
  const int adj = rem < 0 ? -1 : (rem >= d ? 1 : 0);   // selects, no branches
  q = t + adj;
  r = rem - adj * d;
}

// BK pixels per K-step, NS LDS stages (NS - 1 K-steps of DMA in flight ahead of the MFMAs)
template <int WM, int WN, int BK, int NS>
struct WdCfg {
  static constexpr int BMw = 64 * WM, BNw = 64 * WN;          // dY cols (Kout), X cols (T*C)
  static constexpr int RPI_A = 1024 / (BMw * 2), RPI_B = 1024 / (BNw * 2);   // rows / 1-KB DMA
  static constexpr int IA = BK / RPI_A / 4, IB = BK / RPI_B / 4;             // DMAs per wave
  static constexpr int STAGE = BK * (BMw + BNw);                             // bf16 per stage
  static constexpr int LDO = BNw + 4;
  // BK 32 variants stage the fp32 epilogue tile in two row halves (-> ~34-40 KB of LDS, up to
  // 4 blocks per CU with the <= 128-VGPR build)
  static constexpr int EPI_PASSES = BK == 32 ? 2 : 1;
  static constexpr size_t EPI = (size_t)(BMw / EPI_PASSES) * LDO * 4;
  static constexpr size_t LDS = (size_t)(NS * STAGE * 2) > EPI ? (size_t)(NS * STAGE * 2) : EPI;
  static_assert(IA >= 1 && IB >= 1 && BK % 32 == 0, "wgrad DMA plan");
};

// DENSE: one tap at (0, 0), unit stride, P = H, Q = W (see conv_wgrad_pp_kernel): X rows are
// the pixels, no decode / shuffles
template <int WM, int WN, int BK, int NS, bool DENSE = false>
__global__ void __launch_bounds__(kThreads, (BK == 32 && NS == 2) ? 4 : 2)
conv_wgrad_dma_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                      float* __restrict__ dW, const WgradGeom g, const TapTableW taps,
                      float invQ, float invP) {
  using Cf = WdCfg<WM, WN, BK, NS>;
  constexpr int BMw = Cf::BMw, BNw = Cf::BNw;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int TC = taps.n * g.C;
  const int tiles_m = (g.Kout + BMw - 1) / BMw;
  const int tiles_n = (TC + BNw - 1) / BNw;
  const int ntiles = tiles_m * tiles_n;
  // XCD-aware: consecutive logical ids (same split, neighbouring tiles -> the same pixel rows of
  // X / dY) share an XCD's L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntiles;
  const int split = bid / ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int k0 = tm * BMw, j0 = tn * BNw;
  const int M = g.N * g.P * g.Q;
  const int ms = split * (int)g.m_per_split;
  const int me = min(ms + (int)g.m_per_split, M);
  const int nk = (me - ms + BK - 1) / BK;
  const int PQ = g.P * g.Q;                 // split-relative descriptors (see conv_wgrad_kernel)
  const int n_lo = ms / PQ, n_hi = max(n_lo, (me - 1) / PQ);
  const long img = (long)g.H * g.W * g.C;
  const i32x4_t rx = DENSE ? rsrc_quad(X + (long)ms * g.C, (uint32_t)max(me - ms, 0) * g.C * 2u)
                           : rsrc_quad(X + n_lo * img, (uint32_t)((n_hi - n_lo + 1) * img * 2));
  const i32x4_t ry = rsrc_quad(dY + (long)ms * g.Kout, (uint32_t)max(me - ms, 0) * g.Kout * 2u);
  const uint32_t lds0 = lds_addr(lds);
  // tap table -> LDS (read once below, before any DMA reuses the space) so per-lane lookups
  // never index the kernarg struct
  int* lds_taps = reinterpret_cast<int*>(lds);
  if (tid == 0)
    for (int t = 0; t < taps.n; ++t) { lds_taps[t] = taps.dh[t]; lds_taps[DTF_MAX_TAPS + t] = taps.dw[t]; }
  __syncthreads();

  // DMA plan: per stage the dY image is 64 / RPI_A wave-instructions of RPI_A rows, the X image
  // 64 / RPI_B; wave w issues instructions q = w + 4i of each.  Per lane everything that does not
  // change with the K-step is precomputed: the dY column / row offset and the X tap offset and
  // tap displacement of the chunk it fetches.
  int rowa[Cf::IA], a_off[Cf::IA], rowb[Cf::IB], b_dh[Cf::IB], b_dw[Cf::IB], b_toff[Cf::IB];
#pragma unroll
  for (int i = 0; i < Cf::IA; ++i) {
    const int r = Cf::RPI_A * (wave + 4 * i) + lane / (BMw / 8);
    rowa[i] = r;
    const int chunk = (lane % (BMw / 8)) ^ wswz<BMw * 2>(r);
    const int kc = k0 + chunk * 8;
    a_off[i] = kc < g.Kout ? (r * g.Kout + kc) * 2 : -1;
  }
#pragma unroll
  for (int i = 0; i < Cf::IB; ++i) {
    const int r = Cf::RPI_B * (wave + 4 * i) + lane / (BNw / 8);
    rowb[i] = r;
    const int chunk = (lane % (BNw / 8)) ^ wswz<BNw * 2>(r);
    const int jc = j0 + chunk * 8;
    if (DENSE) {
      b_dh[i] = b_dw[i] = 0;
      b_toff[i] = jc < TC ? jc * 2 : -1;
    } else if (jc < TC) {
      const int t = jc / g.C;
      const int c = jc - t * g.C;
      b_dh[i] = lds_taps[t];
      b_dw[i] = lds_taps[DTF_MAX_TAPS + t];
      b_toff[i] = ((b_dh[i] * g.W + b_dw[i]) * g.C + c) * 2;
    } else {
      b_dh[i] = 1 << 20;          // fails the bounds test -> zeros
      b_dw[i] = 0;
      b_toff[i] = 0;
    }
  }
  __syncthreads();                // the tap table is dead: stage 0 may now be filled
  const int HW = g.H * g.W;

  // Each lane decodes ONE pixel of the K-step (row = lane); the lanes that fetch a row's chunks
  // get its decode by ds_bpermute -- one divmod pair per lane per step.
  auto issue = [&](int kt, int stage) {
    const uint32_t base = lds0 + (uint32_t)(stage * Cf::STAGE) * 2u;
    const int mk = ms + kt * BK;                     // wave-uniform first pixel of the step
    const int live = me - mk;                         // rows < live are inside this split
    int pb = 0, hw = 0;
    if (!DENSE) {
      const int mp = mk + lane;
      int t, q, n, p;
      fdivmod(mp < me ? mp : mk, g.Q, invQ, t, q);
      fdivmod(t, g.P, invP, n, p);
      const int hb = lane < live ? p * g.sh : 0x3FFF;   // an invalid row fails every bounds test
      const int wb = q * g.sw;
      pb = (((n - n_lo) * HW + hb * g.W + wb) * g.C) * 2;
      hw = (hb << 16) | wb;
    }
    const uint32_t a_base = (uint32_t)(mk - ms) * g.Kout * 2u;
#pragma unroll
    for (int i = 0; i < Cf::IA; ++i) {
      const int r = rowa[i];
      const uint32_t ao = (r < live && a_off[i] >= 0) ? a_base + (uint32_t)a_off[i] : kOOB;
      dma16(ry, base + (uint32_t)(wave + 4 * i) * 1024u, ao);
    }
#pragma unroll
    for (int i = 0; i < Cf::IB; ++i) {
      const int r = rowb[i];
      if (DENSE) {
        const uint32_t bo = (r < live && b_toff[i] >= 0)
                                ? (uint32_t)(mk - ms + r) * g.C * 2u + (uint32_t)b_toff[i] : kOOB;
        dma16(rx, base + (uint32_t)(BK * BMw * 2) + (uint32_t)(wave + 4 * i) * 1024u, bo);
        continue;
      }
      const int hwr = __shfl(hw, r, 64);
      const int pbr = __shfl(pb, r, 64);
      const int h = (hwr >> 16) + b_dh[i], w = (hwr & 0xFFFF) + b_dw[i];
      const bool bok = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      const uint32_t bo = bok ? (uint32_t)(pbr + b_toff[i]) : kOOB;
      dma16(rx, base + (uint32_t)(BK * BMw * 2) + (uint32_t)(wave + 4 * i) * 1024u, bo);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int gq = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  // NS-stage ring: step k's DMAs were issued NS - 1 steps earlier; steps past nk are issued too,
  // fully out of range (no traffic), so every wait below leaves exactly (NS - 2) steps in flight
  constexpr int PER = Cf::IA + Cf::IB;     // DMAs per wave per step
#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0) issue(s0, s0);
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (NS == 2) {
      DTF_WAIT_VM(0);
      __syncthreads();         // everyone's step kt landed; everyone finished reading kt - 1
    } else {
      static_assert(NS != 3 || PER == 4 || PER == 8 || PER == 10, "vmcnt literal table");
      if constexpr (NS == 4 && PER == 4) DTF_WAIT_VM(8);
      else if constexpr (NS == 4 && PER == 5) DTF_WAIT_VM(10);
      else if constexpr (NS == 3 && PER == 4) DTF_WAIT_VM(4);
      else if constexpr (NS == 3 && PER == 5) DTF_WAIT_VM(5);
      else if constexpr (NS == 3 && PER == 8) DTF_WAIT_VM(8);
      else if constexpr (NS == 3 && PER == 10) DTF_WAIT_VM(10);
      else static_assert(NS == 2, "no vmcnt literal for this pipeline");
      raw_barrier();           // no vmcnt(0) drain: the younger stages stay in flight
    }
    issue(kt + NS - 1, (kt + NS - 1) % NS);
    const bf16_t* sa = lds + (kt % NS) * Cf::STAGE;
    const bf16_t* sb = sa + BK * BMw;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8_t af[4], bfr[4];
      const int r0 = 32 * ks + 8 * gq + tq;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c0 = wm * 64 + 16 * i + 4 * tp;
        const s4_t lo = tr_read(sa + lds_el<BMw>(r0, c0));
        const s4_t hi = tr_read(sa + lds_el<BMw>(r0 + 4, c0));
        af[i] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c0 = wn * 64 + 16 * j + 4 * tp;
        const s4_t lo = tr_read(sb + lds_el<BNw>(r0, c0));
        const s4_t hi = tr_read(sb + lds_el<BNw>(r0 + 4, c0));
        bfr[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  DTF_WAIT_VM(0);
  __syncthreads();             // all fragment reads done before the epilogue reuses the LDS
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  constexpr int LDO = Cf::LDO;
  constexpr int HR = BMw / Cf::EPI_PASSES;          // tile rows staged per pass
  float* so = reinterpret_cast<float*>(lds);
  float* out = dW + (long)split * g.slab;
#pragma unroll
  for (int pass = 0; pass < Cf::EPI_PASSES; ++pass) {
    if (pass) __syncthreads();                      // previous half fully read
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * 64 + 16 * i + 4 * gq + r - pass * HR;
          if (row >= 0 && row < HR)
            so[row * LDO + wn * 64 + 16 * j + li] = acc[i][j][r] + 0.0f;
        }
    __syncthreads();
    for (int idx = tid; idx < HR * BNw; idx += kThreads) {
      const int r = idx / BNw, c = idx % BNw;
      const int row = k0 + pass * HR + r, col = j0 + c;
      if (row < g.Kout && col < TC) out[(long)row * g.ldw + col] = so[r * LDO + c];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Ping-pong wgrad for the compute-bound shapes (Kout >= 256 and T*C >= 256: the 3x3 convs of
// stages 2-4, the late 1x1 convs, every dense layer of BERT): 256 x 256 tile, 8 waves as
// 2 (Kout) x 4 (T*C) of 128 x 64, 64-pixel K-steps in two 64-KB LDS slots.  The schedule is the
// GEMM's (gemm.hip SCHED 2): each K-step is 4 phases {fragment tr-reads | one 16-KB LDS-DMA
// piece (2 per thread) | counted vmcnt | barrier | 16 MFMAs | barrier}, the wm = 1 waves one
// barrier behind the wm = 0 waves, so on every SIMD one wave computes while the other loads.
//   phase:  q0 = (pixels 0-31, Kout top half)   q1 = (0-31, bottom)
//           q2 = (pixels 32-63, top)            q3 = (32-63, bottom)
//   reads:  q0: B(ks0) + A-top(ks0)  q1: A-bottom(ks0)  q2: B(ks1) + A-top(ks1)  q3: A-bottom(ks1)
//   pieces (rows = pixels, row-contiguous 16 KB):  K-step t+1's dY[0:32] at q0, X[0:32] at q1,
//           dY[32:64] at q2, X[32:64] at q3
// RAW: a half is waited (vmcnt(4): the 2 youngest pieces may fly) in the phase before its first
// reader (q1 for the step's second half, q3 for the next step's first), ahead of that phase's
// first barrier.  WAR: every half is restaged >= 3 phases after its last read.
// LDS image rows are 512 B (256 bf16), chunk-swizzled with wswz<512> on the DMA source side.
constexpr int kPpT = 512;
constexpr int kPpBK = 64;                   // pixels per K-step
constexpr int kPpW = 256;                   // operand image width (elements)
constexpr int kPpImg = kPpBK * kPpW;        // one operand image per slot (32 KB)
constexpr int kPpStage = 2 * kPpImg;        // dY image + X image
constexpr int kPpLDO = 260;                 // fp32 epilogue pitch (floats)
constexpr size_t kPpLDS = (size_t)128 * kPpLDO * 4 > (size_t)2 * kPpStage * 2
                              ? (size_t)128 * kPpLDO * 4 : (size_t)2 * kPpStage * 2;
// DEEP: 32-pixel K-steps in a 5-slot ring (32 KB per slot, the whole 160 KB), each step's two
// pieces issued 3 steps ahead -- ~1.5x the latency cover of the 2 x 64-pixel double buffer (an
// L2-resident probe of the latter runs 18-23 % faster, profiles/measurements/r5_wgrad_l2_probe.jsonl).
// Per step: p0 {B + A-top reads | dY piece of step t+3 | barrier | 16 MFMAs | barrier},
// p1 {A-bottom reads | X piece of step t+3 | vmcnt(8): step t+1 landed | barrier | 16 MFMAs |
// barrier}.  WAR: slot (t+3) % 5 was last read in step t-2.  Same MFMA order: bit-identical.
constexpr int kPpDeepBK = 32, kPpDeepSlots = 5;
constexpr int kPpDeepImg = kPpDeepBK * kPpW, kPpDeepStage = 2 * kPpDeepImg;
constexpr size_t kPpDeepLDS = (size_t)kPpDeepSlots * kPpDeepStage * 2;
static_assert(kPpDeepLDS <= 160 * 1024 && kPpDeepLDS >= (size_t)128 * kPpLDO * 4, "deep LDS");

// DENSE: a 1x1 / stride-1 / unpadded conv or a dense layer (one tap at (0, 0), P = H, Q = W):
// pixel m IS row m of X, so the B pieces are addressed like the A pieces -- no per-step pixel
// decode and no cross-lane shuffles (two ds_bpermute per B DMA instruction) in the main loop
// FORM 0: lane-per-pixel decode shuffled to the DMA rows; 1: DENSE; 2: DIRECT per-row decode;
// 4: the lane-per-pixel decode moved to the DMA rows by v_readlane (a DMA instruction's 64 lanes
// fetch only two pixel rows, 2 (wave + 8 j) + {0, 1}: two wave-uniform reads and a select
// instead of a ds_bpermute through the LDS pipe per value)
// SCH 0: the schedule above; 1: DEEP (below); 2: EARLY -- the same 2 x 64-pixel slots with each
// piece issued as soon as its half-slot's WAR margin (2 phases) allows: during step t,
// q0: step t+1 X[0:32], q1: t+1 dY[32:64], q2: t+1 X[32:64], q3: t+2 dY[0:32]; the RAW waits
// (q1: this step's second half, q3: the next step's first) then leave 3 pieces in flight
// (vmcnt(6)), so a piece has 3-5 phases to land instead of 2-3
template <int FORM, int SCH = 0>
__global__ void __launch_bounds__(kPpT, 1)
conv_wgrad_pp_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                     float* __restrict__ dW, const WgradGeom g, const TapTableW taps,
                     float invQ, float invP) {
  // FORM 3 (timing probe only, wrong results): DENSE with every K-step re-reading the split's
  // first 64 rows (L2-resident operands)
  constexpr bool DENSE = FORM == 1 || FORM == 3, DIRECT = FORM == 2, READL = FORM == 4;
  constexpr bool DEEP = SCH == 1, EARLY = SCH == 2;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int TC = taps.n * g.C;
  const int tiles_m = (g.Kout + 255) / 256, tiles_n = (TC + 255) / 256;
  const int ntiles = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int k0 = tm * 256, j0 = tn * 256;
  const int M = g.N * g.P * g.Q;
  const int ms = split * (int)g.m_per_split;
  const int me = min(ms + (int)g.m_per_split, M);
  constexpr int BKS = DEEP ? kPpDeepBK : kPpBK;
  constexpr int STG = DEEP ? kPpDeepStage : kPpStage, IMG = DEEP ? kPpDeepImg : kPpImg;
  const int nk = (me - ms + BKS - 1) / BKS;
  const int PQ = g.P * g.Q;                 // split-relative descriptors (see conv_wgrad_kernel)
  const int n_lo = ms / PQ, n_hi = max(n_lo, (me - 1) / PQ);
  const long img = (long)g.H * g.W * g.C;
  const i32x4_t rx = DENSE ? rsrc_quad(X + (long)ms * g.C, (uint32_t)max(me - ms, 0) * g.C * 2u)
                           : rsrc_quad(X + n_lo * img, (uint32_t)((n_hi - n_lo + 1) * img * 2));
  const i32x4_t ry = rsrc_quad(dY + (long)ms * g.Kout, (uint32_t)max(me - ms, 0) * g.Kout * 2u);
  const uint32_t lds0 = lds_addr(lds);
  int* lds_taps = reinterpret_cast<int*>(lds);
  if (tid == 0)
    for (int t = 0; t < taps.n; ++t) { lds_taps[t] = taps.dh[t]; lds_taps[DTF_MAX_TAPS + t] = taps.dw[t]; }
  __syncthreads();
  // DMA plan: instruction j (0, 1) of a piece fills image rows 2 (wave + 8 j) + {0, 1} of the
  // 32-row half; lane l fetches row (l >> 5)'s logical chunk (l & 31) ^ swizzle
  int a_off[2], b_dh[2], b_dw[2], b_toff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rr = 2 * (wave + 8 * j) + (lane >> 5);
    const int chunk = (lane & 31) ^ wswz<512>(rr);
    const int kc = k0 + chunk * 8;
    a_off[j] = kc < g.Kout ? kc * 2 : -1;
    const int jc = j0 + chunk * 8;
    if (DENSE) {
      b_dh[j] = b_dw[j] = 0;
      b_toff[j] = jc < TC ? jc * 2 : -1;
    } else if (jc < TC) {
      const int t = jc / g.C, c = jc - t * g.C;
      b_dh[j] = lds_taps[t];
      b_dw[j] = lds_taps[DTF_MAX_TAPS + t];
      b_toff[j] = ((b_dh[j] * g.W + b_dw[j]) * g.C + c) * 2;
    } else {
      b_dh[j] = 1 << 20;
      b_dw[j] = 0;
      b_toff[j] = 0;
    }
  }
  __syncthreads();                          // the tap table is dead: slot 0 may now be filled
  const int HW = g.H * g.W;
  // pixel decode of the K-step being issued: lane l holds pixel mk + l's base offset / (h, w)
  // (shuffled to the DMA rows), or with DIRECT each lane decodes the 4 rows it fetches itself
  int dec_pb = 0, dec_hw = 0, dec_live = 0;
  int drow_pb[2][2], drow_hw[2][2];
  auto decode = [&](int kt) {
    const int mk = FORM == 3 ? ms : ms + kt * BKS;
    dec_live = me - mk;
    if (DENSE) return;
    if (DIRECT) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int R = 32 * h + 2 * (wave + 8 * j) + (lane >> 5);
          int t, q, n, p;
          fdivmod(R < dec_live ? mk + R : ms, g.Q, invQ, t, q);
          fdivmod(t, g.P, invP, n, p);
          const int hb = R < dec_live ? p * g.sh : 0x3FFF;
          const int wb = q * g.sw;
          drow_pb[h][j] = (((n - n_lo) * HW + hb * g.W + wb) * g.C) * 2;
          drow_hw[h][j] = (hb << 16) | wb;
        }
      return;
    }
    const int mp = mk + lane;
    int t, q, n, p;
    fdivmod(mp < me ? mp : ms, g.Q, invQ, t, q);
    fdivmod(t, g.P, invP, n, p);
    const int hb = lane < dec_live ? p * g.sh : 0x3FFF;   // an invalid row fails every test
    const int wb = q * g.sw;
    dec_pb = (((n - n_lo) * HW + hb * g.W + wb) * g.C) * 2;
    dec_hw = (hb << 16) | wb;
  };
  // piece pc: 0 = dY rows 0-31, 1 = X rows 0-31, 2 = dY rows 32-63, 3 = X rows 32-63
  auto issue = [&](int kt, int pc) {
    const int h = DEEP ? 0 : pc >> 1;
    const bool isB = pc & 1;
    const int mk = FORM == 3 ? ms : ms + kt * BKS;
    const int slot = DEEP ? kt % kPpDeepSlots : kt & 1;
    const uint32_t base = lds0 + (uint32_t)((slot * STG + (isB ? IMG : 0) + h * 32 * kPpW) * 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int R = 32 * h + 2 * (wave + 8 * j) + (lane >> 5);   // pixel row of the K-step
      const uint32_t dst = base + (uint32_t)(2 * (wave + 8 * j) * kPpW * 2);
      if (!isB) {
        const uint32_t off = (R < dec_live && a_off[j] >= 0)
                                 ? (uint32_t)(mk - ms + R) * g.Kout * 2u + (uint32_t)a_off[j] : kOOB;
        dma16(ry, dst, off);
      } else if (DENSE) {
        const uint32_t off = (R < dec_live && b_toff[j] >= 0)
                                 ? (uint32_t)(mk - ms + R) * g.C * 2u + (uint32_t)b_toff[j] : kOOB;
        dma16(rx, dst, off);
      } else {
        int hwr, pbr;
        if constexpr (DIRECT) {
          hwr = drow_hw[h][j];
          pbr = drow_pb[h][j];
        } else if constexpr (READL) {
          const int R0 = 32 * h + 2 * (wave + 8 * j);            // wave-uniform
          const int hw0 = __builtin_amdgcn_readlane(dec_hw, R0);
          const int hw1 = __builtin_amdgcn_readlane(dec_hw, R0 + 1);
          const int pb0 = __builtin_amdgcn_readlane(dec_pb, R0);
          const int pb1 = __builtin_amdgcn_readlane(dec_pb, R0 + 1);
          hwr = (lane >> 5) ? hw1 : hw0;
          pbr = (lane >> 5) ? pb1 : pb0;
        } else {
          hwr = __shfl(dec_hw, R, 64);
          pbr = __shfl(dec_pb, R, 64);
        }
        const int hh = (hwr >> 16) + b_dh[j], ww = (hwr & 0xFFFF) + b_dw[j];
        const bool ok = (unsigned)hh < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
        dma16(rx, dst, ok ? (uint32_t)(pbr + b_toff[j]) : kOOB);
      }
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const int gq = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  bf16x8_t fA[4], fB[4];
  auto rdA = [&](const bf16_t* sa, int ks, int half) {
    const int r0 = 32 * ks + 8 * gq + tq;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c0 = wm * 128 + half * 64 + 16 * i + 4 * tp;
      const s4_t lo = tr_read(sa + lds_el<kPpW>(r0, c0));
      const s4_t hi = tr_read(sa + lds_el<kPpW>(r0 + 4, c0));
      fA[i] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  auto rdB = [&](const bf16_t* sb, int ks) {
    const int r0 = 32 * ks + 8 * gq + tq;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c0 = wn * 64 + 16 * j + 4 * tp;
      const s4_t lo = tr_read(sb + lds_el<kPpW>(r0, c0));
      const s4_t hi = tr_read(sb + lds_el<kPpW>(r0 + 4, c0));
      fB[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    raw_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_phase = [&](int half) {
    sync();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[half * 4 + i][j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(fA[i], fB[j], acc[half * 4 + i][j], 0, 0, 0);
    sync();
  };

  if constexpr (DEEP) {
#pragma unroll
    for (int s0 = 0; s0 < 3; ++s0) { decode(s0); issue(s0, 0); issue(s0, 1); }
    DTF_WAIT_VM(8);                         // step 0 landed (steps 1, 2 in flight)
    sync();
    if (wm == 1) sync();                    // the one-barrier stagger
    for (int kt = 0; kt < nk; ++kt) {
      const bf16_t* sa = lds + (kt % kPpDeepSlots) * STG;
      const bf16_t* sb = sa + IMG;
      rdB(sb, 0);
      rdA(sa, 0, 0);
      decode(kt + 3);
      issue(kt + 3, 0);
      mfma_phase(0);
      rdA(sa, 0, 1);
      issue(kt + 3, 1);
      DTF_WAIT_VM(8);                       // step kt + 1 landed (kt + 2, kt + 3 in flight)
      mfma_phase(1);
    }
  } else if constexpr (EARLY) {
    decode(0);
    issue(0, 0); issue(0, 1); issue(0, 2); issue(0, 3);
    decode(1);
    issue(1, 0);
    DTF_WAIT_VM(6);                         // step 0's first half landed
    sync();
    if (wm == 1) sync();                    // the one-barrier stagger
    for (int kt = 0; kt < nk; ++kt) {
      const bf16_t* sa = lds + (kt & 1) * kPpStage;
      const bf16_t* sb = sa + kPpImg;
      rdB(sb, 0);
      rdA(sa, 0, 0);
      issue(kt + 1, 1);
      mfma_phase(0);                        // q0
      rdA(sa, 0, 1);
      issue(kt + 1, 2);
      DTF_WAIT_VM(6);                       // this step's second half landed
      mfma_phase(1);                        // q1
      rdB(sb, 1);
      rdA(sa, 1, 0);
      issue(kt + 1, 3);
      mfma_phase(0);                        // q2
      rdA(sa, 1, 1);
      decode(kt + 2);
      issue(kt + 2, 0);
      DTF_WAIT_VM(6);                       // the next step's first half landed
      mfma_phase(1);                        // q3
    }
  } else {
  decode(0);
  issue(0, 0); issue(0, 1); issue(0, 2); issue(0, 3);
  DTF_WAIT_VM(4);                           // step 0's first half landed
  sync();
  if (wm == 1) sync();                      // the one-barrier stagger
  for (int kt = 0; kt < nk; ++kt) {
    const bf16_t* sa = lds + (kt & 1) * kPpStage;
    const bf16_t* sb = sa + kPpImg;
    rdB(sb, 0);
    rdA(sa, 0, 0);
    decode(kt + 1);
    issue(kt + 1, 0);
    mfma_phase(0);                          // q0
    rdA(sa, 0, 1);
    issue(kt + 1, 1);
    DTF_WAIT_VM(4);                         // this step's second half landed
    mfma_phase(1);                          // q1
    rdB(sb, 1);
    rdA(sa, 1, 0);
    issue(kt + 1, 2);
    mfma_phase(0);                          // q2
    rdA(sa, 1, 1);
    issue(kt + 1, 3);
    DTF_WAIT_VM(4);                         // the next step's first half landed
    mfma_phase(1);                          // q3
  }
  }
  if (wm == 0) sync();                      // re-align the barrier counts
  DTF_WAIT_VM(0);                           // the trailing no-op pieces still target the slots
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  float* so = reinterpret_cast<float*>(lds);
  float* out = dW + (long)split * g.slab;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {    // the wm == pass waves stage their 128 rows
    if (pass) __syncthreads();
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            so[(16 * i + 4 * gq + r) * kPpLDO + wn * 64 + 16 * j + li] = acc[i][j][r] + 0.0f;
    }
    __syncthreads();
    for (int idx = tid; idx < 128 * 64; idx += kPpT) {
      const int r = idx >> 6, c4 = idx & 63;
      const int row = k0 + pass * 128 + r, col = j0 + c4 * 4;
      if (row < g.Kout && col < TC)
        *reinterpret_cast<float4*>(out + (long)row * g.ldw + col) =
            *reinterpret_cast<const float4*>(so + r * kPpLDO + c4 * 4);
    }
  }
}

// Deterministic slab sum: block = (256 / G) float4 columns x G split groups; group q sums splits
// q, q+G, ... in order (4 loads in flight per lane), the G group partials are added in a fixed
// order through LDS.  G = 16 for small slabs with many splits (the halo wgrad's 64 x 576 slab x
// 256 blocks: 576 blocks instead of 144 latency-bound ones), else 4.
template <int G>
__global__ void __launch_bounds__(256)
slab_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out, long n, long slab,
                   int nsplit, int accumulate) {
  constexpr int CB = 256 / G;
  __shared__ float4 red[G][CB];
  const int col = threadIdx.x % CB, q = threadIdx.x / CB;
  const long n4 = n >> 2;
  const long i = (long)blockIdx.x * CB + col;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    const float4* base = reinterpret_cast<const float4*>(ws) + i;
    const long s4 = slab >> 2;
    int k = q;
    for (; k + 3 * G < nsplit; k += 4 * G) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = base[(long)(k + u * G) * s4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; k < nsplit; k += G) {
      const float4 v = base[(long)k * s4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[q][col] = s;
  __syncthreads();
  if (q == 0 && i < n4) {
    float4 t = red[0][col];
    for (int k = 1; k < G; ++k) {
      t.x += red[k][col].x; t.y += red[k][col].y; t.z += red[k][col].z; t.w += red[k][col].w;
    }
    if (accumulate) {   // gradient written straight into the optimizer's flat fp32 grad buffer
      const float4 o = reinterpret_cast<const float4*>(out)[i];
      t.x += o.x; t.y += o.y; t.z += o.z; t.w += o.w;
    }
    reinterpret_cast<float4*>(out)[i] = t;
  }
}

// slabs of n floats (n % 4 == 0) at stride `slab` -> out
void launch_slab_reduce(const float* ws, float* out, long n, long slab, int nsplit, int accumulate,
                        hipStream_t st) {
  const long n4 = n / 4;
  if (nsplit >= 32 && (n4 + 63) / 64 < 512)
    hipLaunchKernelGGL(slab_reduce_kernel<16>, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st,
                       ws, out, n, slab, nsplit, accumulate);
  else
    hipLaunchKernelGGL(slab_reduce_kernel<4>, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st,
                       ws, out, n, slab, nsplit, accumulate);
}

// ---------------------------------------------------------------------------------------------
// Halo wgrad for the 56 x 56 x 64 -> 64 3x3 stride-1 convs (ResNet-50 stage 1).  The tiled
// kernels gather every tap's X rows from L2 per output-column tile (~1.5 KB of L2 -> LDS per
// pixel, L2-bound at ~0.35 of the MFMA roof).  Here a block walks whole strips of kHwTH output
// rows: the strip's dY rows and the (kHwTH + 2)-row X patch (zero halo columns) are LDS-DMA'd
// once (double-buffered: the next strip streams in under this strip's MFMAs), and the 9 waves
// each own one tap: dW[:, tap, :] (64 x 64 = 16 fragments in registers) accumulates over every
// strip the block visits.  The tap's B fragments are the patch rows of 8 consecutive output
// pixels shifted by (dh, dw) -- 8 consecutive patch rows, read with the same transposed
// ds_read_b64_tr_b16 pairs as the tiled kernels.  Each block leaves one fp32 slab (64 x 576);
// slab_reduce sums the G slabs in order (deterministic).
constexpr int kHwTH = 4, kHwW = 56, kHwC = 64;
constexpr int kHwT = 9 * 64;                                   // threads: one wave per tap
constexpr int kHwDy = kHwTH * kHwW;                            // dY rows (pixels) per strip
constexpr int kHwPW = kHwW + 2;                                // patch row width
constexpr int kHwPx = (kHwTH + 2) * kHwPW;                     // patch pixels (348)
constexpr int kHwPxAl = (kHwPx + 7) / 8 * 8;                   // DMA-rounded (8 rows / 1 KB)
constexpr int kHwStage = (kHwDy + kHwPxAl) * kHwC;             // elements per stage
constexpr size_t kHwLDS = (size_t)2 * kHwStage * 2;

__global__ void __launch_bounds__(kHwT, 1)
conv_wgrad_halo_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                       float* __restrict__ ws, int N, int H) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // = tap (dh, dw) = (w/3-1, w%3-1)
  const int dh = wave / 3 - 1, dw = wave % 3 - 1;
  const int tiles_h = H / kHwTH;
  const int nstrip = N * tiles_h;
  const int G = gridDim.x;
  const uint32_t lds0 = lds_addr(lds);
  const long img = (long)H * kHwW * kHwC;                      // elements per image
  // X / dY descriptors span the whole tensors (checked < 2^31 bytes on the host)
  const i32x4_t rx = rsrc_quad(X, (uint32_t)((long)N * img * 2));
  const i32x4_t ry = rsrc_quad(dY, (uint32_t)((long)N * img * 2));

  // DMA plan per stage: dY 28 instructions (8 pixels of 128 B each), patch 44; 72 = 8 per wave
  auto issue = [&](int strip, int stage) {
    const bool live = strip < nstrip;
    const int sn = live ? strip / tiles_h : 0, h0 = live ? (strip % tiles_h) * kHwTH : 0;
    const uint32_t base = lds0 + (uint32_t)(stage * kHwStage) * 2u;
    const int rloc = lane >> 3, slot = lane & 7;
    for (int q = wave; q < kHwDy / 8 + kHwPxAl / 8; q += 9) {
      const bool isdy = q < kHwDy / 8;
      const int r = (isdy ? q : q - kHwDy / 8) * 8 + rloc;           // LDS row of the image
      const int chunk = slot ^ wswz<128>(r);
      uint32_t off = kOOB;
      if (isdy) {
        if (live) off = (uint32_t)(((long)sn * img + ((long)h0 * kHwW + r) * kHwC + chunk * 8) * 2);
      } else if (live && r < kHwPx) {
        const int pr = r / kHwPW, pc = r - pr * kHwPW;
        const int h = h0 - 1 + pr, w = pc - 1;
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)kHwW)
          off = (uint32_t)(((long)sn * img + ((long)h * kHwW + w) * kHwC + chunk * 8) * 2);
      }
      dma16(isdy ? ry : rx, base + (uint32_t)(q * 1024), off);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const int gq = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;

  int s = blockIdx.x, it = 0;
  issue(s, 0);
  for (; s < nstrip; s += G, ++it) {
    DTF_WAIT_VM(0);            // this strip's DMAs (own) landed ...
    __syncthreads();           // ... everyone's; everyone finished reading the other stage
    issue(s + G, (it + 1) & 1);                 // past the end: out of range, no traffic
    const bf16_t* sy = lds + (it & 1) * kHwStage;
    const bf16_t* sx = sy + kHwDy * kHwC;
#pragma unroll 1
    for (int kc = 0; kc < kHwDy / 32; ++kc) {
      const int px0 = 32 * kc + 8 * gq;                        // this lane group's 8 pixels
      const int orow = px0 / kHwW, ocol = px0 - orow * kHwW;   // 8 | 56: one output row
      const int pr0 = (orow + 1 + dh) * kHwPW + ocol + 1 + dw;   // their tap-shifted patch rows
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c0 = 16 * i + 4 * tp;
        const s4_t lo = tr_read(sy + lds_el<64>(px0 + tq, c0));
        const s4_t hi = tr_read(sy + lds_el<64>(px0 + tq + 4, c0));
        af[i] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c0 = 16 * j + 4 * tp;
        const s4_t lo = tr_read(sx + lds_el<64>(pr0 + tq, c0));
        const s4_t hi = tr_read(sx + lds_el<64>(pr0 + tq + 4, c0));
        bfr[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  DTF_WAIT_VM(0);              // the trailing no-op DMAs still target the LDS
  // slab of this block: ws[blockIdx.x][k][tap * 64 + c]
  float* out = ws + (long)blockIdx.x * (64 * 576);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(long)(16 * i + 4 * gq + r) * 576 + wave * 64 + 16 * j + li] = acc[i][j][r];
}

// ---------------------------------------------------------------------------------------------
// Halo wgrad for the ResNet-50 stem on its space-to-depth image: a 4 x 4 stride-1 VALID conv,
// X [N][115][115][16] -> dY [N][112][112][64], dW [64][4][4][16] (ops.reference
// space_to_depth_operands).  The tiled kernel gathers each pixel's 16 taps x 32 B from L2
// (512 B of L2 -> LDS traffic per pixel beside its 128 B of dY: 1.23 ms per step at b1984,
// 0.38 PF on the stem's real FLOPs).  Here a block walks strips of kStTH output rows: the strip's
// dY rows and the kStTH + 3 X rows under them -- each one contiguous span -- are LDS-DMA'd once,
// double-buffered (the next strip streams in under this strip's MFMAs).  Wave w owns tap row
// dh = w % 4, i.e. dW[:, dh, 0..3, :] = 64 x 64 (16 fragments), over the strip's 32-pixel chunks
// of parity w / 4 (flipped every strip so both halves do the same number); its B fragment for
// tap (dh, dw) is 2 x 4 consecutive output pixels' X pixels shifted by (dh, dw) -- 32-B rows at a
// 32-B pitch, read with the same transposed ds_read_b64_tr_b16 pairs as the A (dY) fragments.
// The two halves' partial dW meet in LDS in fixed order; each block leaves one fp32 slab
// [64][256], summed in order by slab_reduce (deterministic).
constexpr int kStTH = 2, kStQ = 112, kStXW = 115, kStC = 16, kStK = 64;
constexpr int kStT = 512;                                       // 8 waves: 4 tap rows x 2 halves
constexpr int kStDyB = kStTH * kStQ * kStK * 2;                 // dY bytes per strip (28 KB)
constexpr int kStXB = (kStTH + 3) * kStXW * kStC * 2;           // X bytes per strip (18,400)
constexpr int kStXI = (kStXB + 1023) / 1024;                    // its 1-KB DMA instructions
constexpr int kStStage = kStDyB + kStXI * 1024;                 // bytes per stage
constexpr size_t kStLDS = 2 * (size_t)kStStage;
static_assert(kStLDS >= 4 * 64 * 64 * 4, "the halves' combine area fits the stages");
static_assert(kStQ % 4 == 0 && (kStTH * kStQ) % 32 == 0, "4-pixel groups inside one row");
// K order of a 32-pixel chunk: lane group g takes pixels 4g .. 4g + 3 (lo half of its operand)
// and 16 + 4g .. 16 + 4g + 3 (hi half), the same in both operands, so the two 16-lane groups of a
// 32-lane read pass touch 8 consecutive pixels: 256 contiguous B of the X image (32-B pixels)
// and dY rows 8 apart under this swizzle -- both conflict-free
DTF_DEV int st_swz(int r) { return ((r >> 1) & 3) << 1; }
DTF_DEV int st_el(int r, int c) { return r * 64 + (((c >> 3) ^ st_swz(r)) << 3) + (c & 7); }

// FZ: dY is not a tensor but formed on load -- the stem's BN + ReLU + 3x3/2 max-pool backward
// (pool3s2_bn_bwd_kernel<true>'s arithmetic, bit for bit: pool3s2_gather, the ReLU mask from
// fmaf(x, fsc, fsh), bn_bwd_dx, bf16 rounding) from the pooled gradient, its argmax bytes and the
// BN input x, so that pass never writes d(conv output) (3.2 GB at b1984) nor does this kernel
// read it back.  The strip's x rows are LDS-DMA'd into its dY image (the DMA the unfused kernel
// spends on dY); thread t < 448 owns the 2 x 2 pixel block (column t / 8, 8-channel group t % 8)
// of the strip's block row, whose pooled gradients / argmax bytes for strip s + G it loads into
// registers under strip s's MFMAs, and turns x into dY in place at the top of the strip.
struct StemDz {
  const bf16_t* dp;           // d(pool output) [N][56][56][64]
  const uint8_t* arg;         // its argmax bytes (window position) [N][56][56][64]
  const bf16_t* x;            // the BN input (the stem conv output) [N][112][112][64]
  const float* ca;            // BN backward coefficients: dx = ca dz + cb x + cc
  const float* cb;
  const float* cc;
  const float* fsc;           // forward BN scale / shift (the ReLU mask)
  const float* fsh;
};
constexpr int kStPq = kStQ / 2;                                  // pooled rows / columns (56)

template <bool FZ>
__global__ void __launch_bounds__(kStT, 1)
conv_wgrad_stem_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                       float* __restrict__ ws, int N, const StemDz z) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int dh = wave & 3, half = wave >> 2;
  constexpr int tiles_h = kStQ / kStTH;
  const int nstrip = N * tiles_h;
  const int G = gridDim.x;
  const uint32_t lds0 = lds_addr(lds);
  constexpr long ximg = (long)kStXW * kStXW * kStC;             // elements per image
  constexpr long yimg = (long)kStQ * kStQ * kStK;

  // per stage: dY 28 instructions (8 pixels x 128 B, chunk-swizzled like the 3x3 halo kernel),
  // then X 18 (a flat copy of the strip's contiguous rows); descriptors based at the strip (the
  // tensors pass 2^31 bytes), sized 0 past the last strip (no traffic)
  auto issue = [&](int strip, int stage) {
    const bool live = strip < nstrip;
    const int sn = live ? strip / tiles_h : 0, p0 = live ? (strip % tiles_h) * kStTH : 0;
    const i32x4_t ry = rsrc_quad((FZ ? z.x : dY) + sn * yimg + (long)p0 * kStQ * kStK,
                                 live ? kStDyB : 0);
    const i32x4_t rx = rsrc_quad(X + sn * ximg + (long)p0 * kStXW * kStC, live ? kStXB : 0);
    const uint32_t base = lds0 + (uint32_t)(stage * kStStage);
    const int rloc = lane >> 3, slot = lane & 7;
    for (int q = wave; q < kStDyB / 1024 + kStXI; q += 8) {
      if (q < kStDyB / 1024) {
        // FZ: the BN input x rows (the same [N][112][112][64] layout) land where dY would; the
        // formation pass turns them into dY in place
        const int r = q * 8 + rloc;
        const int chunk = slot ^ st_swz(r);
        dma16(ry, base + (uint32_t)(q * 1024), (uint32_t)((r * kStK + chunk * 8) * 2));
      } else {
        const int qx = q - kStDyB / 1024;
        dma16(rx, base + (uint32_t)(q * 1024), (uint32_t)(qx * 1024 + lane * 16));
      }
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  const int gq = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;

  // FZ operands of this thread's pixel block (registers: loaded one strip ahead)
  const int zb = tid >> 3, zcg = tid & 7;
  const bool zon = FZ && tid < kStPq * 8;
  float za[8], zbb[8], zc[8], zsc[8], zsh[8];
  uint4 zdy[4];
  uint2 zam[4];
  if constexpr (FZ) {
    auto ld8 = [&](const float* p, float* v) {
      const float4 lo = reinterpret_cast<const float4*>(p + zcg * 8)[0];
      const float4 hi = reinterpret_cast<const float4*>(p + zcg * 8)[1];
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z;
      v[7] = hi.w;
    };
    ld8(z.ca, za); ld8(z.cb, zbb); ld8(z.cc, zc); ld8(z.fsc, zsc); ld8(z.fsh, zsh);
  }
  auto zload = [&](int strip) {
    if (!zon || strip >= nstrip) return;
    const uint32_t n = (uint32_t)(strip / tiles_h), a = (uint32_t)(strip % tiles_h);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // pool3s2_bn_bwd_kernel's clamped addresses (P = Q = 56, H = W = 112)
      const uint32_t p = min(a + (k >> 1), (uint32_t)kStPq - 1);
      const uint32_t q = min((uint32_t)zb + (k & 1), (uint32_t)kStPq - 1);
      const uint32_t o = ((n * kStPq + p) * kStPq + q) * 8 + zcg;
      zdy[k] = reinterpret_cast<const uint4*>(z.dp)[o];
      zam[k] = reinterpret_cast<const uint2*>(z.arg)[o];
    }
  };
  auto zform = [&](int strip, bf16_t* sy) {
    if (!zon || strip >= nstrip) return;
    float g[4][8];
    pool3s2_gather(zdy, zam, strip % tiles_h, zb, kStPq, kStPq, g);
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int r = ii * kStQ + 2 * zb + jj;                   // pixel of the 2-row strip
        uint4* slot = reinterpret_cast<uint4*>(sy + st_el(r, zcg * 8));
        float xv[8], o[8];
        unpack8(*slot, xv);                                      // x, DMA'd into the dY image
        const float* gk = g[ii * 2 + jj];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = __builtin_fmaf(xv[e], zsc[e], zsh[e]) > 0.f ? gk[e] : 0.f;
          o[e] = bn_bwd_dx(za[e], d, zbb[e], xv[e], zc[e]);
        }
        *slot = pack8(o);                                        // ... replaced by its dY
      }
  };

  int s = blockIdx.x, it = 0;
  if constexpr (FZ) zload(s);
  issue(s, 0);
  for (; s < nstrip; s += G, ++it) {
    DTF_WAIT_VM(0);            // this strip's DMAs (own) landed ...
    // FZ: form this strip's dY in its stage (last read two trips ago, before the previous
    // trip's barrier)
    if constexpr (FZ) zform(s, lds + (it & 1) * (kStStage / 2));
    __syncthreads();           // ... everyone's; everyone finished reading the other stage
    if constexpr (FZ) zload(s + G);
    issue(s + G, (it + 1) & 1);
    const bf16_t* sy = lds + (it & 1) * (kStStage / 2);
    const bf16_t* sx = sy + kStDyB / 2;
    // (measured: a 3-slot ring, a 2-chunk register double buffer and the same loop unrolled all
    // ran this kernel 0-12 % slower -- r6x2..r6x4)
#pragma unroll 1
    for (int kc = (half + it) & 1; kc < kStTH * kStQ / 32; kc += 2) {
      const int pl = 32 * kc + 4 * gq, ph = pl + 16;            // this lane group's 2 x 4 pixels
      const int rl = pl / kStQ, rh = ph / kStQ;                 // 4 | 112: each 4 in one row
      const int xl = (rl + dh) * kStXW + pl - rl * kStQ;        // X pixels of tap (dh, 0)
      const int xh = (rh + dh) * kStXW + ph - rh * kStQ;
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c0 = 16 * i + 4 * tp;
        const s4_t lo = tr_read(sy + st_el(pl + tq, c0));
        const s4_t hi = tr_read(sy + st_el(ph + tq, c0));
        af[i] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {                             // j = dw
        const s4_t lo = tr_read(sx + (xl + tq + j) * kStC + 4 * tp);
        const s4_t hi = tr_read(sx + (xh + tq + j) * kStC + 4 * tp);
        bfr[j] = (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  DTF_WAIT_VM(0);              // the trailing no-op DMAs still target the LDS
  __syncthreads();             // every fragment read done: the stages become the combine area
  float* red = reinterpret_cast<float*>(lds);                   // [dh][k][64 columns]
  if (half == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          red[(dh * 64 + 16 * i + 4 * gq + r) * 64 + 16 * j + li] = acc[i][j][r];
  }
  __syncthreads();
  if (half == 0) {
    // slab of this block: ws[blockIdx.x][k][(dh * 4 + dw) * 16 + c], half 0 + half 1
    float* out = ws + (long)blockIdx.x * (kStK * 256);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = 16 * i + 4 * gq + r;
          out[(long)k * 256 + dh * 64 + 16 * j + li] =
              acc[i][j][r] + red[(dh * 64 + k) * 64 + 16 * j + li];
        }
  }
}
}  // namespace

// -1 / 1: LDS-DMA kernel whenever legal (default), 0: the register-staged kernel (A/B tests)
static int g_wgrad_dma_mode = -1;
void dtf_wgrad_set_dma_mode(int mode) { g_wgrad_dma_mode = mode; }
// LDS-DMA pipeline: 0 = 64-pixel steps double-buffered; 1 = 32-pixel steps in a 4-stage ring
// (-0.8 % vs 0); 2 = 64-pixel steps, 3 stages, 1 block/CU (-5.6 %); 3 (default) = 32-pixel steps
// double-buffered with a two-pass epilogue: ~34-40 KB of LDS and <= 128 VGPRs -> 4 blocks/CU
// (+1.1 % step vs 0; same-box A/B, profiles/measurements/r1_ab_wgrad_*.txt)
static int g_wgrad_pp = 1;        // ping-pong 256 x 256 kernel for Kout >= 256, T*C >= 256
static int g_wgrad_pp_rounds = 1; // its split-K target: this many rounds of 256 blocks
void dtf_wgrad_set_pp(int v) {
  g_wgrad_pp = v > 0;
  if (v > 0) g_wgrad_pp_rounds = v;
}
// ping-pong kernel: the DENSE form (no pixel decode) for one-tap unit-stride unpadded layers
static int g_wgrad_dense = 1;
void dtf_wgrad_set_dense(int v) { g_wgrad_dense = v; }
// multi-tap / strided layers' pixel decode (A/B knob): 0 lane-per-pixel decode shuffled to the
// DMA rows; 1 each lane decodes the rows it fetches (-0.5..+3 % on stage-3 layers, -10..-15 % on
// stage-4 ones: r5_wgrad_direct_decode_ab.jsonl); 2 the shuffles replaced by v_readlane (15 %
// faster on the stage-3 3x3 layers standalone, -6..+2 % on stage 4, the network -0.2 %:
// r5_wgrad_readlane_decode_ab.jsonl)
static int g_wgrad_direct = 0;
// ping-pong wgrad schedule: 0 the 2 x 64-pixel double buffer, 1 the DEEP 5-slot ring (see
// kPpDeepSlots), 2 EARLY piece issue (conv_wgrad_pp_kernel SCH).  A/B knob, default 0: standalone
// (operands streamed from HBM) EARLY is 9-11 % faster on BERT qkv / ffn1 and DEEP 10-30 % slower;
// in the network (operands just written, MALL-resident) EARLY is neutral: BERT 1.430-1.433M vs
// 1.435M tok/s, ResNet-50 +0.3 % (profiles/measurements/r5_wgrad_schedule_ab.jsonl)
static int g_wgrad_deep = 0;
void dtf_wgrad_set_deep(int v) { g_wgrad_deep = v; }
void dtf_wgrad_set_direct(int v) { g_wgrad_direct = v; }
static bool wgrad_pp(int Kout, int TC) { return g_wgrad_pp && Kout >= 256 && TC >= 256; }
static int g_wgrad_pipe = 3;
void dtf_wgrad_set_pipe(int p) { g_wgrad_pipe = p; }
int dtf_wgrad_get_pipe() { return g_wgrad_pipe; }
// 1 x 4 waves (64 x 256 tile) for multi-tap Kout <= 64 layers (stage-1 3x3, the stem): the 2 x 2
// tile would leave half its MFMA rows empty.  Measured (tools/wgrad_ab.sh, b512): stem 611 ->
// 493 us, 3x3 337 -> 288 us, but the bandwidth-bound 1x1 layers are 11-20 % slower with it, so
// they keep 2 x 2.  Mode 2 disables it (A/B tests).
static bool wgrad_narrow(int Kout, int taps) {
  return g_wgrad_dma_mode != 2 && Kout <= 64 && taps > 1;
}

// Number of reduction splits: aim for ~1024 blocks (4 per CU), keep >= 4 K-steps per split and
// the fp32 slab workspace (splits x Kout x TC) under `ws_cap` floats.
static int g_wgrad_halo = 1;   // stage-1 3x3 wgrad on the halo kernel (0: tiled kernels)
void dtf_wgrad_set_halo(int v) { g_wgrad_halo = v; }
// the halo route: 3x3 stride-1 "same" conv, 56 x 56 x 64 -> 64, standard tap order
static bool wgrad_halo_ok(const WgradGeom& g, const TapTableW& taps) {
  if (!g_wgrad_halo || g.C != kHwC || g.Kout != 64 || g.W != kHwW || g.Q != kHwW || g.P != g.H ||
      g.H % kHwTH || g.sh != 1 || g.sw != 1 || taps.n != 9 || g.ldw != 576 ||
      2.0 * g.N * g.H * g.W * g.C >= 2147483647.0)
    return false;
  for (int t = 0; t < 9; ++t)
    if (taps.dh[t] != t / 3 - 1 || taps.dw[t] != t % 3 - 1) return false;
  return true;
}
// the stem route: the 4 x 4 VALID conv on the s2d image, X 115 x 115 x 16 -> 112 x 112 x 64
static int g_wgrad_stem = 1;   // 0: the tiled kernels (A/B tests)
void dtf_wgrad_set_stem(int v) { g_wgrad_stem = v; }
static bool wgrad_stem_ok(const WgradGeom& g, const TapTableW& taps) {
  if (!g_wgrad_stem || g.C != kStC || g.Kout != kStK || g.H != kStXW || g.W != kStXW ||
      g.P != kStQ || g.Q != kStQ || g.sh != 1 || g.sw != 1 || taps.n != 16 || g.ldw != 256 ||
      g.N <= 0)
    return false;
  for (int t = 0; t < 16; ++t)
    if (taps.dh[t] != t / 4 || taps.dw[t] != t % 4) return false;
  return true;
}
static int wgrad_stem_blocks(int N) {
  const long strips = (long)N * (kStQ / kStTH);
  return strips < 256 ? (int)strips : 256;
}
static int wgrad_halo_blocks(int N, int H) {
  const int strips = N * (H / kHwTH);
  return strips < 256 ? strips : 256;
}
// split count (= fp32 slabs) of the halo route; 0 when it does not apply (Python sizes the
// workspace from this before calling conv_wgrad)
int dtf_conv_wgrad_halo_splits(int N, int H, int W, int C, int P, int Q, int Kout, int sh,
                               int sw, const TapTableW& taps) {
  WgradGeom g{};
  g.N = N; g.H = H; g.W = W; g.C = C; g.P = P; g.Q = Q; g.sh = sh; g.sw = sw; g.Kout = Kout;
  g.ldw = taps.n * C;
  if (wgrad_halo_ok(g, taps)) return wgrad_halo_blocks(N, H);
  return wgrad_stem_ok(g, taps) ? wgrad_stem_blocks(N) : 0;
}

int dtf_conv_wgrad_splits(long M, int Kout, int TC, long ws_cap, int taps) {
  const bool pp = wgrad_pp(Kout, TC);
  const bool nar = !pp && wgrad_narrow(Kout, taps);
  const int bm = pp ? 256 : nar ? 64 : BM, bn = pp ? 256 : nar ? 256 : BN;
  const long tiles = (long)((Kout + bm - 1) / bm) * ((TC + bn - 1) / bn);
  // never overshoot 1024 = exactly two rounds of 512 block slots (2 blocks x 256 CUs): one block
  // past a round costs a whole extra round (29 splits x 36 tiles = 1044 blocks ran 3 rounds);
  // the ping-pong kernel runs one block per CU: two rounds of 256
  long splits = (pp ? 256 * g_wgrad_pp_rounds : 1024) / tiles;
  const long max_splits = (M + 4 * BKM - 1) / (4 * BKM);
  if (splits > max_splits) splits = max_splits;
  const long cap = ws_cap / ((long)Kout * TC);
  if (splits > cap) splits = cap;
  if (splits < 1) splits = 1;
  // normalise so that every split gets work (M rounded to BKM multiples)
  long mps = (M + splits - 1) / splits;
  mps = ((mps + BKM - 1) / BKM) * BKM;
  return (int)((M + mps - 1) / mps);
}

// splits == 1 (and not accumulating): dW written directly.  Otherwise `ws` holds splits x Kout x
// ldw floats; the slabs are summed (in split order) into dW by a second launch, which adds the
// existing dW last when `accumulate` (direct writes into the flat gradient buffer).
void dtf_conv_wgrad(const bf16_t* X, const bf16_t* dY, float* dW, float* ws, WgradGeom g,
                    const TapTableW& taps, int splits, int tr_mode, int accumulate,
                    hipStream_t st) {
  if (taps.n <= 0 || taps.n > DTF_MAX_TAPS) throw std::runtime_error("wgrad: bad tap count");
  if (g.Kout % 8) throw std::runtime_error("wgrad: Kout % 8 != 0");
  const bool via_ws = splits > 1 || accumulate;
  if (splits < 1 || (via_ws && !ws)) throw std::runtime_error("wgrad: bad split workspace");
  if (wgrad_halo_ok(g, taps) && splits == wgrad_halo_blocks(g.N, g.H)) {
    if (!ws) throw std::runtime_error("wgrad halo: needs the slab workspace");
    static bool attr = false;
    if (!attr) {
      HIP_CHECK(hipFuncSetAttribute((const void*)conv_wgrad_halo_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHwLDS));
      attr = true;
    }
    hipLaunchKernelGGL(conv_wgrad_halo_kernel, dim3((unsigned)splits), dim3(kHwT), kHwLDS, st, X,
                       dY, ws, g.N, g.H);
    launch_slab_reduce(ws, dW, 64L * 576, 64L * 576, splits, accumulate, st);
    return;
  }

  if (wgrad_stem_ok(g, taps) && splits == wgrad_stem_blocks(g.N)) {
    if (!ws) throw std::runtime_error("wgrad stem: needs the slab workspace");
    static bool attr = false;
    if (!attr) {
      HIP_CHECK(hipFuncSetAttribute((const void*)conv_wgrad_stem_kernel<false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStLDS));
      attr = true;
    }
    hipLaunchKernelGGL(conv_wgrad_stem_kernel<false>, dim3((unsigned)splits), dim3(kStT), kStLDS,
                       st, X, dY, ws, g.N, StemDz{});
    launch_slab_reduce(ws, dW, (long)kStK * 256, (long)kStK * 256, splits, accumulate, st);
    return;
  }

  const long M = (long)g.N * g.P * g.Q;
  const int TC = taps.n * g.C;
  long mps = (M + splits - 1) / splits;
  mps = ((mps + BKM - 1) / BKM) * BKM;
  // the kernels rebase X / dY at each split's first image / row: one split's span (not the
  // tensor) must fit 32-bit byte offsets
  const double span_imgs = (double)mps / ((double)g.P * g.Q) + 2.0;
  if (M >= 2147483647L || 2.0 * mps * g.Kout >= 2147483647.0 ||
      2.0 * span_imgs * g.H * g.W * g.C >= 2147483647.0)
    throw std::runtime_error("wgrad: split span too large for 32-bit buffer offsets (more splits)");
  g.m_per_split = mps;
  g.slab = (long)g.Kout * g.ldw;
  const int nsplit = (int)((M + mps - 1) / mps);
  if (nsplit != splits) throw std::runtime_error("wgrad: split plan mismatch");
  float* target = via_ws ? ws : dW;
  const size_t lds = (size_t)2 * (OPER_A + OPER_B) * sizeof(bf16_t) + 2 * DTF_MAX_TAPS * sizeof(int);
  const bool generic = (g.C % 8) != 0;
  // fdivmod (float reciprocal + one correction step) is exact while m / Q < 2^21; the DMA
  // kernels pack a pixel's (h, w) as (h << 16) | w
  const bool dma = g_wgrad_dma_mode != 0 && !generic && (tr_mode & 1) && M / g.Q < (1L << 21) &&
                   g.H < 16000 && g.W < 65536;
  const bool narrow = dma && wgrad_narrow(g.Kout, taps.n);
  const int bm = narrow ? 64 : BM, bn = narrow ? 256 : BN;
  const long tiles = (long)((g.Kout + bm - 1) / bm) * ((TC + bn - 1) / bn);
  const dim3 grid((unsigned)(tiles * nsplit));
  const bool dense1 = (g_wgrad_dense & 1) && taps.n == 1 && taps.dh[0] == 0 && taps.dw[0] == 0 &&
                      g.sh == 1 && g.sw == 1 && g.H == g.P && g.W == g.Q;
  if (dma && wgrad_pp(g.Kout, TC) && g.ldw % 4 == 0) {
    static bool attr = false;
    if (!attr) {
      for (const void* k : {(const void*)conv_wgrad_pp_kernel<0>,
                            (const void*)conv_wgrad_pp_kernel<1>,
                            (const void*)conv_wgrad_pp_kernel<2>,
                            (const void*)conv_wgrad_pp_kernel<3>,
                            (const void*)conv_wgrad_pp_kernel<4>,
                            (const void*)conv_wgrad_pp_kernel<0, 2>,
                            (const void*)conv_wgrad_pp_kernel<1, 2>,
                            (const void*)conv_wgrad_pp_kernel<2, 2>,
                            (const void*)conv_wgrad_pp_kernel<3, 2>})
        HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPpLDS));
      for (const void* k : {(const void*)conv_wgrad_pp_kernel<0, 1>,
                            (const void*)conv_wgrad_pp_kernel<1, 1>,
                            (const void*)conv_wgrad_pp_kernel<2, 1>,
                            (const void*)conv_wgrad_pp_kernel<3, 1>})
        HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kPpDeepLDS));
      attr = true;
    }
    const long ptiles = (long)((g.Kout + 255) / 256) * ((TC + 255) / 256);
    const bool deep = g_wgrad_deep == 1;
    const int form = dense1 ? (g_wgrad_dense == 3 ? 3 : 1)
                            : g_wgrad_direct == 1 ? 2 : g_wgrad_direct == 2 ? 4 : 0;
    using PpKern = void (*)(const bf16_t*, const bf16_t*, float*, const WgradGeom, const TapTableW,
                            float, float);
    static const PpKern kerns[3][4] = {
        {conv_wgrad_pp_kernel<0>, conv_wgrad_pp_kernel<1>, conv_wgrad_pp_kernel<2>,
         conv_wgrad_pp_kernel<3>},
        {conv_wgrad_pp_kernel<0, 1>, conv_wgrad_pp_kernel<1, 1>, conv_wgrad_pp_kernel<2, 1>,
         conv_wgrad_pp_kernel<3, 1>},
        {conv_wgrad_pp_kernel<0, 2>, conv_wgrad_pp_kernel<1, 2>, conv_wgrad_pp_kernel<2, 2>,
         conv_wgrad_pp_kernel<3, 2>}};
    const int sch = g_wgrad_deep >= 0 && g_wgrad_deep <= 2 ? g_wgrad_deep : 0;
    auto kern = form == 4 ? conv_wgrad_pp_kernel<4> : kerns[sch][form];
    hipLaunchKernelGGL(kern, dim3((unsigned)(ptiles * nsplit)), dim3(kPpT),
                       deep ? kPpDeepLDS : kPpLDS, st, X, dY, target, g, taps,
                       1.0f / (float)g.Q, 1.0f / (float)g.P);
  } else if (dma) {
    const float iq = 1.0f / (float)g.Q, ip = 1.0f / (float)g.P;
#define DTF_WGRAD_LAUNCH(WM_, WN_, BK_, NS_)                                                     \
  do {                                                                                           \
    if (dense1)                                                                                  \
      hipLaunchKernelGGL((conv_wgrad_dma_kernel<WM_, WN_, BK_, NS_, true>), grid,               \
                         dim3(kThreads), (WdCfg<WM_, WN_, BK_, NS_>::LDS), st, X, dY, target, g, \
                         taps, iq, ip);                                                          \
    else                                                                                         \
      hipLaunchKernelGGL((conv_wgrad_dma_kernel<WM_, WN_, BK_, NS_>), grid, dim3(kThreads),     \
                         (WdCfg<WM_, WN_, BK_, NS_>::LDS), st, X, dY, target, g, taps, iq, ip); \
  } while (0)
    if (g_wgrad_pipe == 1) {   // 32-pixel steps, 4-stage ring (3 steps of DMA in flight)
      if (narrow) DTF_WGRAD_LAUNCH(1, 4, 32, 4);
      else DTF_WGRAD_LAUNCH(2, 2, 32, 4);
    } else if (g_wgrad_pipe == 3) {   // 32-pixel steps, double buffer, half epilogue: 4 blk/CU
      if (narrow) DTF_WGRAD_LAUNCH(1, 4, 32, 2);
      else DTF_WGRAD_LAUNCH(2, 2, 32, 2);
    } else if (g_wgrad_pipe == 2) {   // 64-pixel steps, 3-stage ring (1 block / CU)
      if (narrow) DTF_WGRAD_LAUNCH(1, 4, 64, 3);
      else DTF_WGRAD_LAUNCH(2, 2, 64, 3);
    } else {                   // 64-pixel steps, double buffer
      if (narrow) DTF_WGRAD_LAUNCH(1, 4, 64, 2);
      else DTF_WGRAD_LAUNCH(2, 2, 64, 2);
    }
#undef DTF_WGRAD_LAUNCH
  } else if (!(tr_mode & 1)) {  // debug path: element-wise LDS reads instead of ds_read_b64_tr_b16
    if (generic) hipLaunchKernelGGL((conv_wgrad_kernel<true, false>), grid, dim3(kThreads), lds, st, X, dY, target, g, taps, tr_mode >> 1);
    else hipLaunchKernelGGL((conv_wgrad_kernel<false, false>), grid, dim3(kThreads), lds, st, X, dY, target, g, taps, tr_mode >> 1);
  } else if (generic) {
    hipLaunchKernelGGL((conv_wgrad_kernel<true, true>), grid, dim3(kThreads), lds, st, X, dY, target, g, taps, tr_mode >> 1);
  } else {
    hipLaunchKernelGGL((conv_wgrad_kernel<false, true>), grid, dim3(kThreads), lds, st, X, dY, target, g, taps, tr_mode >> 1);
  }
  if (via_ws) {
    // slab = Kout * ldw floats, Kout % 8 == 0 -> slab % 4 == 0 (float4 path covers it)
    launch_slab_reduce(ws, dW, g.slab, g.slab, nsplit, accumulate, st);
  }
}

// Deterministic sum of `nsplit` contiguous fp32 slabs of n floats (n % 4 == 0) into `out`
// (+= when accumulate): the split-K combine of the dense-layer weight-gradient GEMMs.
void dtf_slab_reduce(const float* ws, float* out, long n, int nsplit, int accumulate, hipStream_t st) {
  if (n % 4) throw std::runtime_error("slab_reduce: n % 4 != 0");
  launch_slab_reduce(ws, out, n, n, nsplit, accumulate, st);
}


// The stem weight gradient with its dY formed on load from the BN + ReLU + max-pool backward's
// operands (conv_wgrad_stem_kernel<true>): X the space-to-depth image [N][115][115][16], dp / arg
// the pooled gradient and argmax bytes [N][56][56][64], xbn the BN input [N][112][112][64],
// (ca, cb, cc) the BN backward coefficients, (fsc, fsh) the forward scale / shift.  dW [64][256]
// fp32 (+= with accumulate), via the [wgrad_stem_blocks(N)][64][256] slab workspace ws.
int dtf_wgrad_stem_dz_splits(int N) { return g_wgrad_stem && N > 0 ? wgrad_stem_blocks(N) : 0; }
void dtf_conv_wgrad_stem_dz(const bf16_t* X, const bf16_t* dp, const uint8_t* arg,
                            const bf16_t* xbn, const float* ca, const float* cb, const float* cc,
                            const float* fsc, const float* fsh, float* dW, float* ws, int N,
                            int accumulate, hipStream_t st) {
  if (N <= 0 || !ws || (long)N * kStQ * kStQ * (kStK / 8) >= 2147483647L)
    throw std::runtime_error("wgrad stem dz: bad batch / workspace");
  const int splits = wgrad_stem_blocks(N);
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)conv_wgrad_stem_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kStLDS));
    hipFuncAttributes fa{};
    HIP_CHECK(hipFuncGetAttributes(&fa, (const void*)conv_wgrad_stem_kernel<true>));
    if (fa.localSizeBytes > 0)
      throw std::runtime_error("conv_wgrad_stem_kernel<true> was compiled with register spills");
    attr = true;
  }
  const StemDz z{dp, arg, xbn, ca, cb, cc, fsc, fsh};
  hipLaunchKernelGGL(conv_wgrad_stem_kernel<true>, dim3((unsigned)splits), dim3(kStT), kStLDS, st,
                     X, nullptr, ws, N, z);
  launch_slab_reduce(ws, dW, (long)kStK * 256, (long)kStK * 256, splits, accumulate, st);
}
