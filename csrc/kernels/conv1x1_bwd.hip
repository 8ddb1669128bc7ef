// Fused backward of ResNet-50's expanding 1x1 convs (c3: C -> K = 4C channels) whose input is
// relu(BN(x)) (ops/native.py _BnReluConv1x1), for the first two stages (C = 64, 128):
//
//   dY[m, c]   = sum_k dO[m, k] W[k, c]                  (data gradient, bf16 out)
//   dW[k, c]  += sum_m dO[m, k] Y[m, c]                  (weight gradient, fp32 slab per block)
//   BN sums[c] = sum_m dz, sum_m dz (x - mean) invstd,   dz = dY * [x sc + sh > 0]
//
// Unfused these are three passes -- the weight-gradient kernel (reads dO, Y), the data-gradient
// GEMM (reads dO, writes dY) and the BN backward's reduce (reads dY, x): 2K + 6C bytes of HBM
// traffic per row (1536 at C = 64).  Here ONE pass reads dO, Y and x and writes dY: 2K + 6C - ...
// = 896 B per row at C = 64; the 4 K C FLOPs per row are a small fraction of what the MFMA pipes
// could do in the time the bytes take, so the kernel is a streaming problem.
// (profiles/measurements/r3_conv_roofline_b1984.jsonl: the dgrad and wgrad passes of the C = 64
// layer alone take 0.75 ms each at batch 1984.)
//
// Design (persistent: one block per CU, TM-row tiles walked with a grid stride):
//   * dO (TM x K), Y (TM x C) and x (TM x C) tiles stream through a 3-slot LDS ring by LDS-DMA,
//     two tiles ahead, with source-side XOR swizzles chosen for the reads below;
//   * data gradient with the operands swapped -- A = W^T rows (the wave's channel blocks, whole
//     K, held in VGPRs for the kernel's lifetime), B = dO rows from LDS -- so every lane ends up
//     with 4 CONSECUTIVE channels of one row: one 8-byte store of dY, one 8-byte LDS read of x
//     for the BN sums (computed on dY exactly as it is stored, like gemm_stream.hip's epilogue);
//   * weight gradient: the wave owns dW rows [K/NW w, K/NW (w + 1)) x all C channels (register
//     accumulators for ALL of the block's tiles: 32 fp32 per lane at C = 64, 128 at C = 128);
//     both operands are read
//     with the hardware transpose read ds_read_b64_tr_b16 (the reduction runs over tile rows);
//   * at the end every block writes one fp32 dW slab [K][C] and one BN slab row [2][C]; the host
//     reduces the slabs in fixed order (deterministic; slab_reduce / bn_bwd_finalize_g).
// Only global memory traffic per tile per wave: D DMA instructions + S dY stores, so the counted
// vmcnt waits at the top of a tile are exact (see `top`).
#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int kNB = 3;               // ring slots

typedef __attribute__((ext_vector_type(4))) short s4_t;
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

// per-shape configuration: C in, K out, TM rows per tile, NW waves; LZ: the conv-output gradient
// dO is formed in the kernel from the consuming BatchNorm's (dy, x3, ReLU bit mask) and its
// backward coefficients (see `LAZY` below) instead of being read
// RC (with LZ): x3 is not read either -- recomputed per tile from Y and W with the forward's exact
// MFMA chain (x3 = bf16(Y W^T), ks in order), so the kernel reads neither dO nor x3
template <int C_, int K_, int TM_, int NW_, bool LZ_ = false, bool RC_ = false>
struct Cfg {
  static constexpr int C = C_, K = K_, TM = TM_, NW = NW_;
  static constexpr bool LZ = LZ_, RC = RC_;
  static constexpr int T = NW * 64;
  static constexpr int NCB = C / 16;                         // channel blocks
  static constexpr int CPW = NCB >= NW ? NCB / NW : 1;       // dgrad channel blocks per wave
  static constexpr int WPC = NW / (NCB / CPW);               // waves sharing a channel block
  static constexpr int MBW = TM / 16 / WPC;                  // dgrad row blocks per wave
  static constexpr int KS = K / 32;                          // dgrad MFMA k-steps
  static constexpr int KBW = K / NW / 16;                    // wgrad dW row blocks per wave
  static constexpr int DO = TM * K;                          // bf16 per dO tile
  static constexpr int YT = TM * C;                          // bf16 per Y / x tile
  static constexpr int OT = (LZ && !RC) ? 2 * DO : DO;      // dO / dy3 tile (+ x3 tile: LZ, !RC)
  static constexpr int MB = LZ ? TM * K / 8 : 0;             // LZ: ReLU mask bytes per tile
  static constexpr int MI = MB / 1024;                       // ... = 1-KB DMAs, by wave 0
  static constexpr int SLOT = OT + 2 * YT + MB / 2;
  static constexpr int DOI = OT * 2 / 1024;                  // 1-KB DMA instructions per dO tile(s)
  static constexpr int YI = YT * 2 / 1024;                   // ... per Y / x tile
  static constexpr int D = (DOI + 2 * YI) / NW;              // DMA instructions per wave per tile
  static constexpr int S = CPW * MBW;                        // dY stores per lane per tile
  static constexpr int MCH = LZ ? TM * K / 8 / T : 0;       // LZ: 8-channel chunks per thread
  static constexpr size_t LDS = (size_t)kNB * SLOT * 2 + (size_t)WPC * 2 * C * 4 + 4 * C * 4 +
                                (LZ ? (size_t)3 * K * 4 : 0);   // LZ: the A / B / C coefficients
  static_assert(!LZ || ((RC || ((TM * K / 8) % T == 0 && T % (K / 8) == 0)) && MB % 1024 == 0 &&
                        MI <= NW), "LZ transform split");
  static_assert(DOI % NW == 0 && (2 * YI) % NW == 0, "DMA split");
  static_assert(WPC * (NCB / CPW) == NW && MBW >= 1 && (TM % 32 == 0 || TM == 16), "wave split");
  static_assert(LDS <= 160 * 1024, "conv1x1_bwd LDS");
};

// 16-B chunk swizzles (physical chunk = logical chunk ^ swz(row)):
//  dO (rows of a multiple of 256 B): the 16 rows of a dgrad B-fragment read (ds_read_b128, 16
//    lanes / pass) hit 16 different 16-B bank slots; the 8 rows of a transpose-read half-wave keep
//    their 32-B column pair adjacent and land on 8 different pairs
DTF_DEV int swz_o(int r) { return 2 * (r & 7) + ((r >> 3) & 1); }
//  Y (transpose reads only: 8 rows x one 32-B pair per half-wave -> 16 distinct slots)
template <int C>
DTF_DEV int swz_y(int r) { return C == 64 ? 2 * ((r >> 1) & 3) : 2 * (r & 7); }
//  x (8-B reads of 16 rows x one 16-B chunk per half-wave)
template <int C>
DTF_DEV int swz_x(int r) { return C == 64 ? (r >> 1) & 7 : r & 15; }

template <int RP>
DTF_DEV int sidx(int r, int c, int s) { return r * RP + (((c >> 3) ^ s) << 3) + (c & 7); }

// 8 reduction rows x one column as an MFMA operand (key permutation: j < 4 -> row0 + 4g + j,
// j >= 4 -> row0 + 16 + 4g + j - 4; the same in both operands of a product)
template <int RP, int C, bool DOUT>
DTF_DEV bf16x8_t tr8(const bf16_t* base, int row0, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int r = row0 + 4 * g + (i >> 2), c = col0 + 4 * (i & 3);
  const int s0 = DOUT ? swz_o(r) : swz_y<C>(r);
  const int s1 = DOUT ? swz_o(r + 16) : swz_y<C>(r + 16);
  const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(base + sidx<RP>(r, c, s0)));
  const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(base + sidx<RP>(r + 16, c, s1)));
  return (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// 4 reduction rows (4g .. 4g + 3 for lane group g) x one column: the 16x16x16 operand
template <int RP, int C, bool DOUT>
DTF_DEV s4_t tr4(const bf16_t* base, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int r = 4 * g + (i >> 2), c = col0 + 4 * (i & 3);
  const int s0 = DOUT ? swz_o(r) : swz_y<C>(r);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(base + sidx<RP>(r, c, s0)));
}

DTF_DEV f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int N>
DTF_DEV void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <class F>
constexpr int RC_KBW() { return F::RC ? F::K / F::NW / 16 : 1; }

struct C1Args {
  const bf16_t* dout;   // [M][K]  gradient of the conv output
  const bf16_t* wt;     // [C][K]  W^T (wt[c][k] = W[k][c])
  const bf16_t* y;      // [M][C]  the conv input relu(BN(x))
  const bf16_t* x;      // [M][C]  the BatchNorm input
  const float* mean;
  const float* inv;
  const float* sc;      // forward scale / shift (ReLU recomputed from x)
  const float* sh;
  bf16_t* dy;           // [M][C]  data gradient (of y)
  float* wpart;         // [grid][K][C]
  float* bpart;         // [grid][2][C]
  int M;
  // LZ: dO = bn_bwd_dx(cA, dy3 * mask bit, cB, x3, cC) per element (the consuming residual
  // BatchNorm's backward apply, never stored); `dout` then holds that BN's incoming gradient dy3
  const bf16_t* x3;     // [M][K]  the BN's input (this conv's output)
  const uint8_t* mask;  // [M][K / 8] ReLU bit mask of the BN's forward
  const float* cA;
  const float* cB;
  const float* cC;
  const bf16_t* w;      // RC: the conv weight [K][C] (x3 = Y W^T)
};

template <class F>
__global__ void __launch_bounds__(F::T, 1) conv1x1_bwd_kernel(const C1Args g) {
  constexpr int C = F::C, K = F::K, TM = F::TM, NW = F::NW;
  constexpr int CPW = F::CPW, MBW = F::MBW, KS = F::KS, KBW = F::KBW, NCB = F::NCB;
  constexpr bool LZ = F::LZ;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  float* sred = reinterpret_cast<float*>(lds + kNB * F::SLOT);   // [WPC][2][C]
  float* sprm = sred + F::WPC * 2 * C;                            // [4][C] mean / inv / sc / sh
  float* scoef = sprm + 4 * C;                                    // LZ: [3][K] A / B / C
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, gq = lane >> 4;
  const int ntiles = g.M / TM;
  const int nmy = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  // data gradient: channel blocks cg * CPW .. + CPW - 1, rows mw * MBW * 16 .. of each tile
  const int cg = wave % (NCB / CPW), mw = wave / (NCB / CPW);

  // W^T fragments: the wave's channel blocks x the whole reduction (loaded once)
  bf16x8_t wf[CPW][KS];
#pragma unroll
  for (int j = 0; j < CPW; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[j][ks] = *reinterpret_cast<const bf16x8_t*>(g.wt + ((cg * CPW + j) * 16 + li) * K +
                                                      ks * 32 + gq * 8);
  for (int t = tid; t < C; t += F::T) {
    sprm[t] = g.mean[t];
    sprm[C + t] = g.inv[t];
    sprm[2 * C + t] = g.sc[t];
    sprm[3 * C + t] = g.sh[t];
  }

  const uint32_t lds0 = lds_addr(lds);
  // tile i of this block -> slot i % 3.  dO: instruction q covers 1024 / (2K) rows; Y / x:
  // 1024 / (2C) rows per instruction
  // LZ issues every tile index (past the block's last tile: out-of-range offsets, the range check
  // drops the reads and the DMA fills a free slot with zeros) so its vmcnt counts are constant
  auto issue = [&](int i) {
    const bool live = !LZ || i < nmy;
    const long m0 = ((long)blockIdx.x + (long)(live ? i : 0) * gridDim.x) * TM;
    const i32x4_t ro = rsrc_quad(g.dout + m0 * K, (uint32_t)(F::DO * 2));
    const i32x4_t r3 = rsrc_quad(LZ ? g.x3 + m0 * K : g.dout, (uint32_t)(F::DO * 2));
    const i32x4_t ry = rsrc_quad(g.y + m0 * C, (uint32_t)(F::YT * 2));
    const i32x4_t rx = rsrc_quad(g.x + m0 * C, (uint32_t)(F::YT * 2));
    const uint32_t base = lds0 + (uint32_t)((i % kNB) * F::SLOT * 2);
    constexpr int OL = K / 8, YL = C / 8;        // 16-B chunks per row
    constexpr int OI1 = F::DO * 2 / 1024;        // instructions per K-wide tile
#pragma unroll
    for (int j = 0; j < F::DOI / NW; ++j) {
      const int q = wave + NW * j;
      const int qq = q % OI1, e = qq * 64 + lane;          // chunk index in the tile
      const int r = e / OL, s = e % OL;
      const uint32_t off = live ? (uint32_t)((r * K + ((s ^ swz_o(r)) << 3)) * 2) : 0xFFFFFFF0u;
      dma16(q < OI1 ? ro : r3, base + (uint32_t)q * 1024u, off);
    }
#pragma unroll
    for (int j = 0; j < 2 * F::YI / NW; ++j) {      // Y instructions 0 .. YI-1, then x
      const int q = wave + NW * j;
      const bool isx = q >= F::YI;
      const int qq = isx ? q - F::YI : q, e = qq * 64 + lane;
      const int r = e / YL, s = e % YL;
      const int sw = isx ? swz_x<C>(r) : swz_y<C>(r);
      const uint32_t off = live ? (uint32_t)((r * C + ((s ^ sw) << 3)) * 2) : 0xFFFFFFF0u;
      dma16(isx ? rx : ry, base + (uint32_t)(F::OT * 2 + q * 1024), off);
    }
    if constexpr (LZ) {             // the tile's mask bytes (row-major, unswizzled): waves < MI
      if (wave < F::MI) {
        const i32x4_t rm = rsrc_quad(g.mask + m0 * (K / 8), (uint32_t)F::MB);
        dma16(rm, base + (uint32_t)((F::OT + 2 * F::YT) * 2 + wave * 1024),
              live ? (uint32_t)(wave * 1024 + lane * 16) : 0xFFFFFFF0u);
      }
    }
  };
  // LZ: this thread's 8-channel chunks of every tile (rows t / (K/8) + k T / (K/8), column chunk
  // t % (K/8)) and the chunk's coefficients
  constexpr int MCH = F::MCH > 0 ? F::MCH : 1;
  if constexpr (LZ) {
    for (int t = tid; t < K; t += F::T) {
      scoef[t] = g.cA[t];
      scoef[K + t] = g.cB[t];
      scoef[2 * K + t] = g.cC[t];
    }
  }
  // RC: W fragments for this wave's x3 columns k in [wave K/NW, (wave+1) K/NW), all C (A operand)
  constexpr int KSC = C / 32;
  bf16x8_t wr[RC_KBW<F>()][KSC];
  float rca[RC_KBW<F>()][4], rcb[RC_KBW<F>()][4], rcc[RC_KBW<F>()][4];   // RC: this lane's A/B/C
  if constexpr (F::RC) {
#pragma unroll
    for (int kb = 0; kb < RC_KBW<F>(); ++kb) {
#pragma unroll
      for (int ks = 0; ks < KSC; ++ks)
        wr[kb][ks] = *reinterpret_cast<const bf16x8_t*>(
            g.w + (long)(wave * (K / NW) + kb * 16 + li) * C + ks * 32 + gq * 8);
      // the 4 columns this lane forms in every tile are fixed: coefficients in registers
      const int k0 = wave * (K / NW) + kb * 16 + 4 * gq;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        rca[kb][r] = g.cA[k0 + r];
        rcb[kb][r] = g.cB[k0 + r];
        rcc[kb][r] = g.cC[k0 + r];
      }
    }
  }

  f32x4_t aw[KBW][NCB];
#pragma unroll
  for (int a = 0; a < KBW; ++a)
#pragma unroll
    for (int b = 0; b < NCB; ++b) aw[a][b] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float s1[CPW][4], s2[CPW][4];
#pragma unroll
  for (int j = 0; j < CPW; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s1[j][e] = s2[j][e] = 0.f;

  constexpr int D = F::D, S = F::S;
  if constexpr (LZ) {
    issue(0);
    issue(1);
  } else {
    issue(0);
    if (nmy > 1) issue(1);
  }
  for (int i = 0; i < nmy; ++i) {
    if constexpr (LZ) {
      // top: tile i's DMAs landed.  Every tile index is issued (constant counts); younger: tile
      // i + 1's DMAs (D, + the mask DMA on waves < MI) and the dY stores of tiles i - 1, i - 2
      if (wave < F::MI) {
        if (i == 0) wait_vm<D + 1>();
        else if (i == 1) wait_vm<D + 1 + S>();
        else wait_vm<D + 1 + 2 * S>();
      } else {
        if (i == 0) wait_vm<D>();
        else if (i == 1) wait_vm<D + S>();
        else wait_vm<D + 2 * S>();
      }
    } else {
      // top: this wave's DMAs of tile i landed.  Younger vector-memory ops at this point: tile
      // i + 1's DMAs (D, if it exists) and the dY stores of tiles i - 1 and i - 2 (S each).
      const bool more = i + 1 < nmy;
      if (i == 0) { if (more) wait_vm<D>(); else wait_vm<0>(); }
      else if (i == 1) { if (more) wait_vm<D + S>(); else wait_vm<S>(); }
      else { if (more) wait_vm<D + 2 * S>(); else wait_vm<2 * S>(); }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();                  // every wave's DMAs landed; slot (i + 2) % 3 was read in i - 1
    if constexpr (LZ) {
      issue(i + 2);
    } else {
      if (i + 2 < nmy) issue(i + 2);
    }
    bf16_t* const slot = lds + (i % kNB) * F::SLOT;
    if constexpr (LZ && F::RC) {
      // x3 of this wave's columns recomputed from Y (the forward stream GEMM's chain with the
      // operands swapped: the same products in the same k order, bit-identical) and dO formed in
      // place over dy3 -- lane (li, gq): row 16 mb + li, columns k0 .. k0 + 3
      int lx = lane;
      asm volatile("" : "+v"(lx));
      const int xi = lx & 15, xq = lx >> 4;
      const uint8_t* msk = reinterpret_cast<const uint8_t*>(slot + F::OT + 2 * F::YT);
#pragma unroll
      for (int mb = 0; mb < TM / 16; ++mb) {
        const int m = mb * 16 + xi;
        bf16x8_t yb[KSC];
#pragma unroll
        for (int ks = 0; ks < KSC; ++ks)
          yb[ks] = *reinterpret_cast<const bf16x8_t*>(slot + F::OT + sidx<C>(m, ks * 32 + xq * 8, swz_y<C>(m)));
#pragma unroll
        for (int kb = 0; kb < RC_KBW<F>(); ++kb) {
          f32x4_t a = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < KSC; ++ks) a = mfma16(wr[kb][ks], yb[ks], a);
          const int k0 = wave * (K / NW) + kb * 16 + 4 * xq;
          const int o = sidx<K>(m, k0, swz_o(m));
          const uint2 d = *reinterpret_cast<const uint2*>(slot + o);
          const uint32_t mbits = (uint32_t)msk[m * (K / 8) + (k0 >> 3)] >> (k0 & 7);
          const float* ca = rca[kb];
          const float* cb = rcb[kb];
          const float* cc = rcc[kb];
          const float gv[4] = {__builtin_bit_cast(float, d.x << 16), __builtin_bit_cast(float, d.x & 0xffff0000u),
                               __builtin_bit_cast(float, d.y << 16), __builtin_bit_cast(float, d.y & 0xffff0000u)};
          float ov[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float xv = bf2f(f2bf(a[r]));          // x3 exactly as the forward stored it
            const float dz = (mbits >> r) & 1u ? gv[r] : 0.f;
            ov[r] = bn_bwd_dx(ca[r], dz, cb[r], xv, cc[r]);
          }
          *reinterpret_cast<uint2*>(slot + o) = make_uint2(pack2(ov[0], ov[1]), pack2(ov[2], ov[3]));
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    } else if constexpr (LZ) {
      // dO = the residual BatchNorm's backward apply, in place over the dy3 tile (bit-identical to
      // bn_bwd_apply_kernel<1>'s stored dx: same dz, same bn_bwd_dx, same bf16 rounding)
      int tt = tid;                 // recomputed per tile (see `ln` below)
      asm volatile("" : "+v"(tt));
      const int lch = tt % (K / 8), lrow = tt / (K / 8);
#pragma unroll
      for (int k = 0; k < MCH; ++k) {
        const int r = lrow + k * (F::T / (K / 8));
        const int o = sidx<K>(r, lch * 8, swz_o(r));
        float gv[8], xv[8], ov[8];
        unpack8(*reinterpret_cast<const uint4*>(slot + o), gv);
        unpack8(*reinterpret_cast<const uint4*>(slot + F::DO + o), xv);
        const uint32_t mb = reinterpret_cast<const uint8_t*>(slot + F::OT + 2 * F::YT)[r * (K / 8) + lch];
        float ca[8], cb[8], cc[8];
        *reinterpret_cast<float4*>(ca) = *reinterpret_cast<const float4*>(scoef + lch * 8);
        *reinterpret_cast<float4*>(ca + 4) = *reinterpret_cast<const float4*>(scoef + lch * 8 + 4);
        *reinterpret_cast<float4*>(cb) = *reinterpret_cast<const float4*>(scoef + K + lch * 8);
        *reinterpret_cast<float4*>(cb + 4) = *reinterpret_cast<const float4*>(scoef + K + lch * 8 + 4);
        *reinterpret_cast<float4*>(cc) = *reinterpret_cast<const float4*>(scoef + 2 * K + lch * 8);
        *reinterpret_cast<float4*>(cc + 4) = *reinterpret_cast<const float4*>(scoef + 2 * K + lch * 8 + 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = (mb >> e) & 1u ? gv[e] : 0.f;
          ov[e] = bn_bwd_dx(ca[e], dz, cb[e], xv[e], cc[e]);
        }
        *reinterpret_cast<uint4*>(slot + o) = pack8(ov);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    }
    const bf16_t* sO = slot;
    const bf16_t* sY = sO + F::OT;
    const bf16_t* sX = sY + F::YT;
    // the swizzled per-lane LDS addresses are recomputed every tile (a few VALU ops each) rather
    // than hoisted out of the loop: at C = 128 the hoisted set does not fit next to the register-
    // resident W^T fragments and dW accumulators and would be spilled
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int li = ln & 15, gq = ln >> 4;

    // data gradient: rows mw * MBW * 16 + 16 f + li, channels of block cg * CPW + j, 4 per lane
    f32x4_t ad[CPW][MBW];
#pragma unroll
    for (int j = 0; j < CPW; ++j)
#pragma unroll
      for (int f = 0; f < MBW; ++f) ad[j][f] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int f = 0; f < MBW; ++f) {
        const int m = (mw * MBW + f) * 16 + li;
        const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(sO + sidx<K>(m, ks * 32 + gq * 8, swz_o(m)));
#pragma unroll
        for (int j = 0; j < CPW; ++j) ad[j][f] = mfma16(wf[j][ks], b, ad[j][f]);
      }
    }
    // weight gradient: dW rows wave * K / NW + 16 kb + .., channels 16 cb + .., over the tile
    if constexpr (TM == 16) {       // 16-deep reduction: v_mfma_f32_16x16x16_bf16, one tr read each
      s4_t fa[KBW];
#pragma unroll
      for (int kb = 0; kb < KBW; ++kb) fa[kb] = tr4<K, C, true>(sO, wave * (K / NW) + kb * 16, ln);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const s4_t fb = tr4<C, C, false>(sY, cb * 16, ln);
#pragma unroll
        for (int kb = 0; kb < KBW; ++kb)
          aw[kb][cb] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(fa[kb], fb, aw[kb][cb], 0, 0, 0);
      }
    }
#pragma unroll
    for (int ms = 0; ms < TM / 32; ++ms) {
      bf16x8_t fa[KBW];
#pragma unroll
      for (int kb = 0; kb < KBW; ++kb) fa[kb] = tr8<K, C, true>(sO, 32 * ms, wave * (K / NW) + kb * 16, ln);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const bf16x8_t fb = tr8<C, C, false>(sY, 32 * ms, cb * 16, ln);
#pragma unroll
        for (int kb = 0; kb < KBW; ++kb) aw[kb][cb] = mfma16(fa[kb], fb, aw[kb][cb]);
      }
    }
    // epilogue: dY (bf16) + the BatchNorm backward sums on the stored values
    const long m0 = ((long)blockIdx.x + (long)i * gridDim.x) * TM;
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int c0 = (cg * CPW + j) * 16 + 4 * gq;
      float mu[4], is[4], sc[4], sh[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mu[e] = sprm[c0 + e];
        is[e] = sprm[C + c0 + e];
        sc[e] = sprm[2 * C + c0 + e];
        sh[e] = sprm[3 * C + c0 + e];
      }
#pragma unroll
      for (int f = 0; f < MBW; ++f) {
        const int m = (mw * MBW + f) * 16 + li;
        const uint2 pk = make_uint2(pack2(ad[j][f][0], ad[j][f][1]), pack2(ad[j][f][2], ad[j][f][3]));
        *reinterpret_cast<uint2*>(g.dy + (m0 + m) * C + c0) = pk;
        const uint2 xr = *reinterpret_cast<const uint2*>(sX + sidx<C>(m, c0, swz_x<C>(m)));
        const float gd[4] = {__builtin_bit_cast(float, pk.x << 16), __builtin_bit_cast(float, pk.x & 0xffff0000u),
                             __builtin_bit_cast(float, pk.y << 16), __builtin_bit_cast(float, pk.y & 0xffff0000u)};
        const float xv[4] = {__builtin_bit_cast(float, xr.x << 16), __builtin_bit_cast(float, xr.x & 0xffff0000u),
                             __builtin_bit_cast(float, xr.y << 16), __builtin_bit_cast(float, xr.y & 0xffff0000u)};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float dz = __builtin_fmaf(xv[e], sc[e], sh[e]) > 0.f ? gd[e] : 0.f;
          s1[j][e] += dz;
          s2[j][e] += dz * (xv[e] - mu[e]) * is[e];
        }
      }
    }
  }
  DTF_WAIT_VM(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();

  // BN partials: the 16 row lanes sharing a channel group meet by cross-lane adds, then the
  // WPC waves sharing a channel block in fixed order
#pragma unroll
  for (int j = 0; j < CPW; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[j][e] += __shfl_xor(s1[j][e], o, 64);
        s2[j][e] += __shfl_xor(s2[j][e], o, 64);
      }
    }
  if (li == 0) {
#pragma unroll
    for (int j = 0; j < CPW; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = (cg * CPW + j) * 16 + 4 * gq + e;
        sred[(mw * 2 + 0) * C + c] = s1[j][e];
        sred[(mw * 2 + 1) * C + c] = s2[j][e];
      }
  }
  __syncthreads();
  for (int t = tid; t < 2 * C; t += F::T) {
    const int which = t / C, col = t % C;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < F::WPC; ++w) v += sred[(w * 2 + which) * C + col];
    g.bpart[((long)blockIdx.x * 2 + which) * C + col] = v;
  }
  // dW slab: lane holds dW[wave K / NW + 16 kb + 4 gq + r][16 cb + li]
  float* wp = g.wpart + (long)blockIdx.x * K * C;
#pragma unroll
  for (int kb = 0; kb < KBW; ++kb)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        wp[(wave * (K / NW) + kb * 16 + 4 * gq + r) * C + cb * 16 + li] = aw[kb][cb][r];
}

typedef Cfg<64, 256, 64, 8> CfgS0;    // stage 0: 56 x 56 x 64 -> 256
typedef Cfg<64, 256, 64, 16> CfgS0W;  // ... as 16 waves (<= 128 VGPRs: 4 waves per SIMD)
typedef Cfg<128, 512, 32, 8> CfgS1;   // stage 1: 28 x 28 x 128 -> 512
typedef Cfg<64, 256, 64, 8, true, true> CfgS0L;   // stage 0, dO formed from the residual BN,
                                                  // x3 recomputed (LZ + RC)
typedef Cfg<64, 256, 64, 16, true, true> CfgS0LW; // ... as 16 waves
typedef Cfg<128, 512, 16, 8, true> CfgS1L;  // stage 1, LZ (16-row tiles: 42 KB ring slots)

int g_c1_grid = 0;   // 0 = one block per CU
int g_c1_w16 = 0;    // stage 0 as 16-wave blocks: 3 % faster alone, 0.4 % slower in the step (A/B)

int c1_tm(int C) { return C == 64 ? CfgS0::TM : CfgS1::TM; }

int c1_blocks_tm(int M, int TM) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int want = g_c1_grid > 0 ? g_c1_grid : cus;
  const int ntiles = M / TM;
  return ntiles < want ? ntiles : want;
}
int c1_blocks(int M, int C) { return c1_blocks_tm(M, c1_tm(C)); }

template <class F>
void launch_c1(const C1Args& g, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)conv1x1_bwd_kernel<F>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)F::LDS));
    attr = true;
  }
  hipLaunchKernelGGL(conv1x1_bwd_kernel<F>, dim3(c1_blocks_tm(g.M, F::TM)), dim3(F::T), F::LDS, st,
                     g);
}

}  // namespace

bool dtf_conv1x1_bwd_ok(int M, int C, int K) {
  return ((C == 64 && K == 256) || (C == 128 && K == 512)) && M > 0 && M % c1_tm(C) == 0;
}

// number of slab rows (blocks) the fused backward writes for M rows of C channels
int dtf_conv1x1_bwd_blocks(int M, int C) {
  if (!dtf_conv1x1_bwd_ok(M, C, 4 * C)) throw std::runtime_error("conv1x1_bwd: shape");
  return c1_blocks(M, C);
}

void dtf_conv1x1_bwd_set_grid(int n) { g_c1_grid = n; }
void dtf_conv1x1_bwd_set_w16(int v) { g_c1_w16 = v; }

void dtf_conv1x1_bwd(const bf16_t* dout, const bf16_t* wt, const bf16_t* y, const bf16_t* x,
                     const float* mean, const float* inv, const float* sc, const float* sh,
                     bf16_t* dy, float* wpart, float* bpart, int M, int C, int K, hipStream_t st) {
  if (!dtf_conv1x1_bwd_ok(M, C, K))
    throw std::runtime_error("conv1x1_bwd: (C, K) in {(64, 256), (128, 512)}, M % tile == 0");
  const void* ptrs[] = {dout, wt, y, x, mean, inv, sc, sh, dy, wpart, bpart};
  for (const void* p : ptrs)
    if (!p || (reinterpret_cast<uintptr_t>(p) & 15))
      throw std::runtime_error("conv1x1_bwd: null or misaligned operand");
  C1Args g{dout, wt, y, x, mean, inv, sc, sh, dy, wpart, bpart, M};
  if (C == 64) {
    if (g_c1_w16) launch_c1<CfgS0W>(g, st);
    else launch_c1<CfgS0>(g, st);
  } else {
    launch_c1<CfgS1>(g, st);
  }
}

// LZ form (stages 0 and 1): the conv-output gradient dO is never stored -- formed per tile from the
// residual BatchNorm's incoming gradient dy3, its input x3, its forward ReLU bit mask and its
// backward coefficients (A, B, C) -- which removes that BN's apply pass write of dO and this
// kernel's read of it (4 B per element of the 256-channel tensor).
bool dtf_conv1x1_bwd_lazy_ok(int M, int C, int K) {
  if (M <= 0) return false;
  if (C == CfgS0L::C && K == CfgS0L::K) return M % CfgS0L::TM == 0;
  if (C == CfgS1L::C && K == CfgS1L::K) return M % CfgS1L::TM == 0;
  return false;
}
int dtf_conv1x1_bwd_lazy_blocks(int M, int C) {
  if (!dtf_conv1x1_bwd_lazy_ok(M, C, 4 * C)) throw std::runtime_error("conv1x1_bwd_lazy: shape");
  return c1_blocks_tm(M, C == 64 ? CfgS0L::TM : CfgS1L::TM);
}
void dtf_conv1x1_bwd_lazy(const bf16_t* dy3, const bf16_t* x3, const uint8_t* mask,
                          const float* cA, const float* cB, const float* cC, const bf16_t* wt,
                          const bf16_t* y, const bf16_t* x, const float* mean, const float* inv,
                          const float* sc, const float* sh, bf16_t* dy, float* wpart,
                          float* bpart, int M, int C, int K, const bf16_t* w, hipStream_t st) {
  if (!dtf_conv1x1_bwd_lazy_ok(M, C, K))
    throw std::runtime_error("conv1x1_bwd_lazy: (C, K) in {(64, 256), (128, 512)}, M % tile == 0");
  const void* ptrs[] = {dy3, x3, mask, cA, cB, cC, wt, y, x, mean, inv, sc, sh, dy, wpart, bpart, w};
  for (const void* p : ptrs)
    if (!p || (reinterpret_cast<uintptr_t>(p) & 15))
      throw std::runtime_error("conv1x1_bwd_lazy: null or misaligned operand");
  C1Args g{dy3, wt, y, x, mean, inv, sc, sh, dy, wpart, bpart, M, x3, mask, cA, cB, cC, w};
  if (C == 64) {
    if (g_c1_w16) launch_c1<CfgS0LW>(g, st);
    else launch_c1<CfgS0L>(g, st);
  } else {
    launch_c1<CfgS1L>(g, st);
  }
}
