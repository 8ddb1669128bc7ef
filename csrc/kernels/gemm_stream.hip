// Row-streaming GEMM for OUTPUT-HEAVY shapes (short reduction, wide output):
//   C[M, N] = A[M, K] . B[N, K]^T   (+ BN statistics | + Cin | + acc_src * relu_bit)
// K in {64, 128, 256}, N % 64 == 0.  In ResNet-50 these are the expanding 1x1 convs (c3: w -> 4w
// forward) and the data gradients of the reducing ones (c1 of the identity blocks: dgrad w -> 4w):
// per element of output they do 2K FLOPs but write 2 B, so a tile kernel alternates a short
// K-loop with a long store phase -- and with one 256 x 256 tile per CU (gemm.hip) or 128 x 128
// tiles whose K-loop is latency-bound (the register conv kernel) the two phases serialise: both
// run these shapes at 2-4 TB/s (profiles/measurements/r3_gemm_occ2_and_epilogue_split.jsonl,
// r2_conv_roofline_b1984.jsonl: 0.48-0.65 of the HBM roof).
//
// Design (one block of 8 waves per CU, 256 output rows per block, walking ALL of N):
//   * each wave owns 32 rows; their A fragments for the whole K (K/4 VGPRs) are loaded ONCE,
//     straight from HBM into MFMA operand registers -- A is never re-read;
//   * B (the weights, L2-resident) streams through a 3-slot LDS ring in 64-column chunks by
//     LDS-DMA (buffer_load ... lds, source-side XOR swizzle: the same conflict-free 64-deep panel
//     layout as gemm.hip), issued two chunks ahead;
//   * per chunk: K/32 x 8 v_mfma_f32_16x16x32_bf16 per wave, then the wave stages its 32 x 64
//     bf16 outputs in a PRIVATE LDS area (no block barrier) and writes them as 16-B row-contiguous
//     stores (8 rows x 128 B per wave-instruction) -- fire-and-forget: the next chunk's MFMAs
//     start at once and the stores drain under them.  One block barrier per chunk (ring reuse).
//   * every lane issues the same number of vector-memory ops per chunk (rows past M get buffer
//     offsets past the descriptor, dropped by the range check), so the counted vmcnt waits are
//     exact: the top of chunk c waits only for ITS B chunk, never for the stores of c-1 / c-2.
//   * BN statistics: per-lane column sums of the bf16-rounded outputs + cross-lane adds; the 8
//     waves' partials meet in LDS and are summed in fixed order into ONE slab row per block
//     ([ceil(M / 256)][2][N], the same slab shape as gemm.hip's, so the BN finalize is shared).
//   * accumulate modes (data gradients): Cin (beta = 1) or the identity-block residual gradient
//     formed from (dy, ReLU bit mask); the chunk's operands are prefetched one chunk ahead.
// Per output element the MFMA sequence (k = 0..31, 32..63, ... in order) is the one gemm.hip
// runs, so C is bit-identical to the ping-pong GEMM (tests/test_gemm_stream_gpu.py).
#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int kST = 512;      // threads: 8 waves
constexpr int kSWR = 32;      // rows per wave
constexpr int kSBM = 256;     // rows per block
constexpr int kSBN = 64;      // output columns per chunk
constexpr int kSP = 72;       // staging row pitch (bf16): 144 B, conflict-free fragment writes
constexpr uint32_t kSOOB = 0x80000000u;

struct StreamArgs {
  const bf16_t* A; const bf16_t* B; bf16_t* C;
  const bf16_t* Cin;          // beta = 1 accumulate source ([M][ldc]) or null
  const bf16_t* acc_src;      // C += acc_src * relu_bit ([M][N], ldc == N) or null
  const uint8_t* acc_mask;
  float* stats;               // [ceil(M/256)][2][N] or null (also the BN-backward slab)
  int M, N, lda, ldb, ldc;
  int nt;
  // BN-backward sums of the BatchNorm whose OUTPUT gradient this GEMM produces (a data gradient):
  // sum dz, sum dz * (x - mean) * invstd per channel, dz = C * relu_bit, into `stats`
  const bf16_t* bx;           // that BN's input x ([M][N], dense)
  const float* bmean;
  const float* binv;
  const float* bsc;           // forward scale / shift (ReLU bit recomputed from x, kind 2)
  const float* bsh;
  const uint8_t* bmask;       // ReLU bit mask (kind 1)
  // PRE: A is the INPUT of a BatchNorm + ReLU (the producing conv's output); the kernel applies
  // y = bf16(max(x * pre_sc[k] + pre_sh[k], 0)) to its A rows in registers -- exactly the BN
  // apply pass's arithmetic -- and writes y to `pre_y` (the weight gradient's operand)
  const float* pre_sc;
  const float* pre_sh;
  bf16_t* pre_y;
  // DUAL (kind 1 only): C is also the output gradient of a second BatchNorm whose output was
  // ADDED before the shared ReLU (a projection block's shortcut BN): its sums sum dz,
  // sum dz * (xp - meanp) * invstdp go to `statsp` ([ceil(M/256)][2][N])
  const bf16_t* bxp;
  const float* bmeanp;
  const float* binvp;
  float* statsp;
  // RC (BNB with K3 > 0): the BatchNorm input x (a conv output that was never stored) is
  // recomputed per chunk as bf16(y2 . w3^T) -- the producing stream GEMM's exact MFMA chain --
  // from y2 [M][K3] (that conv's input) and w3 [N][K3] (its weight)
  const bf16_t* y2;
  const bf16_t* w3;
  // APPLY (MODE 3): C = relu(bf16(A . B^T) * asc[n] + ash[n] + Cin) -- the residual BatchNorm's
  // apply pass on a conv output recomputed instead of read -- and its ReLU bit mask `amask`
  const float* asc;
  const float* ash;
  uint8_t* amask;
  int k3;                     // RC recompute depth
  int nost;                   // PRE: statistics only, C not stored
};

DTF_DEV int sswz(int row, int ch) { return ch ^ ((row >> 1) & 7); }   // 64-deep panel swizzle

DTF_DEV __amdgpu_buffer_rsrc_t srsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// s_waitcnt vmcnt(N), N a compile-time count
template <int N>
DTF_DEV void wait_vmc() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// MODE: 0 plain, 1 + Cin, 2 + acc_src * relu_bit; STATS: BN statistics slab of the output;
// BMK >= 0: BN-backward sums of the output (0 no ReLU, 1 ReLU bit mask, 2 ReLU from x)
// PROBE (timing experiments only, tools/gemm_bench.py --stream-probe): 1 no MFMAs, 2 no LDS
// staging of C, 4 no chunk barrier, 8 C stores out of range
// NOST: C is not stored (statistics only -- a conv output recomputed later, never written);
// K3 > 0 (BNB): the BN input x recomputed per chunk from y2 / w3 (RC above); MODE 3: APPLY
template <int K, int MODE, bool STATS, int BMK = -1, bool PRE = false, int PROBE = 0,
          bool DUAL = false, bool NOST = false, int K3 = 0>
__global__ void __launch_bounds__(kST, 1) gemm_stream_kernel(const StreamArgs g) {
  constexpr int KS = K / 32;                  // MFMA k-steps
  constexpr int KS3 = K3 / 32;                // RC: recompute k-steps
  constexpr int CHB = kSBN * K;               // bf16 elements of a ring slot's B chunk
  constexpr int CH = CHB + kSBN * K3;         // ... + the RC w3 chunk
  constexpr int D = K / 64 + K3 / 64;         // LDS-DMA instructions per thread per chunk
  constexpr int S = kSWR * kSBN * 2 / (64 * 16);   // 16-B stores per lane per chunk (4)
  // vector-memory stores per lane per chunk: C (+ the APPLY mask bytes); none with NOST
  constexpr int SST = NOST ? 0 : (MODE == 3 ? 2 * S : S);
  static_assert(K3 == 0 || (BMK == 1 && !DUAL), "RC: the residual BatchNorm's bit-mask kind");
  static_assert(MODE != 3 || (!STATS && BMK < 0 && !PRE), "APPLY: a plain epilogue");
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  bf16_t* stg = lds + 3 * CH;
  static_assert(!DUAL || BMK == 1, "DUAL: the residual BatchNorm's ReLU bit mask");
  constexpr int NQ = DUAL ? 3 : 2;                                 // per-channel quantities
  float* sred = reinterpret_cast<float*>(stg + 8 * kSWR * kSP);   // [2][8][NQ][64]
  float* bprm = sred + 2 * 8 * NQ * kSBN;   // BNB: [4][N] mean/inv/sc/sh (DUAL: mean/inv/meanp/invp)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fq = lane >> 4;
  const long m0 = (long)blockIdx.x * kSBM;
  const int rows_blk = (int)min((long)kSBM, (long)g.M - m0);
  const int nch = g.N / kSBN;
  constexpr bool BNB = BMK >= 0;
  static_assert(!(STATS && BNB), "one slab per launch");
  constexpr bool do_stats = STATS || BNB;
  constexpr int mode = MODE;
  // prefetch loads per chunk: the accumulate operands (APPLY: the residual), the BN input (not
  // with RC: recomputed), its mask bytes
  constexpr int L = (MODE == 1 || MODE == 3 ? S : (MODE == 2 ? 2 * S : 0)) +
                    (BNB && K3 == 0 ? S : 0) + (BMK == 1 ? S : 0) + (DUAL ? S : 0);

  // BNB: this block's copy of the per-channel parameters (one float4 per array per thread:
  // N <= 2048), written to LDS after the first wait
  constexpr int NPRM = (BMK == 2 || DUAL) ? 4 : 2;
  float4 prm[NPRM];
  constexpr bool HASPRM = BNB || MODE == 3;     // per-channel parameters staged in LDS
  if constexpr (HASPRM) {
    const float* arrs[4] = {MODE == 3 ? g.asc : g.bmean, MODE == 3 ? g.ash : g.binv,
                            DUAL ? g.bmeanp : g.bsc, DUAL ? g.binvp : g.bsh};
#pragma unroll
    for (int a = 0; a < NPRM; ++a)
      prm[a] = tid * 4 < g.N ? *reinterpret_cast<const float4*>(arrs[a] + tid * 4)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // A: this wave's 32 rows x K, straight into MFMA operand registers
  const __amdgpu_buffer_rsrc_t ra =
      srsrc(g.A + m0 * g.lda, (uint32_t)(((long)(rows_blk - 1) * g.lda + K) * 2));
  bf16x8_t af[2][KS];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = wave * kSWR + i * 16 + frow;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint32_t off = r < rows_blk ? (uint32_t)((r * g.lda + ks * 32 + fq * 8) * 2) : kSOOB;
      af[i][ks] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
    }
  }

  // RC: this wave's 32 rows of y2 (the recompute's A operand), loaded once like A
  constexpr int KS3R = KS3 > 0 ? KS3 : 1;
  bf16x8_t yf[2][KS3R];
  if constexpr (K3 > 0) {
    const __amdgpu_buffer_rsrc_t ry2 =
        srsrc(g.y2 + m0 * K3, (uint32_t)(((long)(rows_blk - 1) * K3 + K3) * 2));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wave * kSWR + i * 16 + frow;
#pragma unroll
      for (int ks = 0; ks < KS3; ++ks) {
        const uint32_t off = r < rows_blk ? (uint32_t)((r * K3 + ks * 32 + fq * 8) * 2) : kSOOB;
        yf[i][ks] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(ry2, off, 0, 0));
      }
    }
  }

  // B chunk c -> ring slot c % 3: DMA instruction q = wave + 8 j fills rows (q % 8) * 8 .. + 7 of
  // 64-deep panel q / 8; chunks past the end are issued too, out of range (constant counts).
  // RC: the slot's second part holds the w3 chunk (rows c * 64 .., K3 deep), same layout
  const i32x4_t rb = rsrc_quad(g.B, (uint32_t)(((long)(g.N - 1) * g.ldb + K) * 2));
  const i32x4_t rw3 = rsrc_quad(K3 > 0 ? (const void*)g.w3 : (const void*)g.B,
                                K3 > 0 ? (uint32_t)((long)g.N * K3 * 2) : 0u);
  const uint32_t lds0 = lds_addr(lds);
  const int lrow = lane >> 3, slot = lane & 7;
  auto issue = [&](int c) {
    const bool live = c < nch;
    const uint32_t base = lds0 + (uint32_t)((c % 3) * CH) * 2u;
#pragma unroll
    for (int j = 0; j < K / 64; ++j) {
      const int q = wave + 8 * j, kp = q >> 3, rg = q & 7;
      const int r = rg * 8 + lrow;
      const uint32_t off = live ? (uint32_t)(((c * kSBN + r) * g.ldb + kp * 64 + sswz(r, slot) * 8) * 2)
                                : 0xFFFFFFF0u;
      dma16(rb, base + (uint32_t)(kp * 64 * 64 + rg * 8 * 64) * 2u, off);
    }
#pragma unroll
    for (int j = 0; j < K3 / 64; ++j) {
      const int q = wave + 8 * j, kp = q >> 3, rg = q & 7;
      const int r = rg * 8 + lrow;
      const uint32_t off = live ? (uint32_t)(((c * kSBN + r) * K3 + kp * 64 + sswz(r, slot) * 8) * 2)
                                : 0xFFFFFFF0u;
      dma16(rw3, base + (uint32_t)(CHB + kp * 64 * 64 + rg * 8 * 64) * 2u, off);
    }
  };

  // epilogue addressing: lane -> rows t * 8 + lane / 8 (t < 4) of the wave's 32, 16-B chunk lane % 8
  const long ldc = g.ldc;
  const __amdgpu_buffer_rsrc_t rc = srsrc(g.C + m0 * ldc, (uint32_t)(rows_blk * ldc * 2));
  const __amdgpu_buffer_rsrc_t rcin =
      srsrc(mode == 1 || mode == 3 ? (const void*)(g.Cin + m0 * ldc)
                                   : (const void*)(g.acc_src + m0 * ldc),
            mode ? (uint32_t)(rows_blk * ldc * 2) : 0u);
  const __amdgpu_buffer_rsrc_t ramask =
      srsrc(mode == 3 ? (const void*)(g.amask + m0 * ldc / 8) : (const void*)g.C,
            mode == 3 ? (uint32_t)(rows_blk * ldc / 8) : 0u);
  const __amdgpu_buffer_rsrc_t rmask =
      srsrc(mode == 2 ? (const void*)(g.acc_mask + m0 * ldc / 8) : (const void*)g.C,
            mode == 2 ? (uint32_t)(rows_blk * ldc / 8) : 0u);
  const int er = lane >> 3, ec = lane & 7;
  auto eoff = [&](int t, int c) -> uint32_t {     // byte offset of (row, chunk) in C / Cin
    const int rr = wave * kSWR + t * 8 + er;
    return rr < rows_blk ? (uint32_t)((rr * ldc + c * kSBN + ec * 8) * 2) : kSOOB;
  };
  uint4 pre[S], bxp[S], bpp[S];
  uint32_t pmask[S], bmp[S];
  const __amdgpu_buffer_rsrc_t rbx =
      srsrc(BNB && K3 == 0 ? (const void*)(g.bx + m0 * ldc) : (const void*)g.C,
            BNB ? (uint32_t)(rows_blk * ldc * 2) : 0u);
  const __amdgpu_buffer_rsrc_t rbm =
      srsrc(BMK == 1 ? (const void*)(g.bmask + m0 * ldc / 8) : (const void*)g.C,
            BMK == 1 ? (uint32_t)(rows_blk * ldc / 8) : 0u);
  const __amdgpu_buffer_rsrc_t rbp =
      srsrc(DUAL ? (const void*)(g.bxp + m0 * ldc) : (const void*)g.C,
            DUAL ? (uint32_t)(rows_blk * ldc * 2) : 0u);
  auto prefetch = [&](int c) {
    if constexpr (L == 0) return;
    const int cc = c < nch ? c : 0;
#pragma unroll
    for (int t = 0; t < S; ++t) {
      const uint32_t off = eoff(t, cc);
      if constexpr (MODE != 0)
        pre[t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rcin, off, 0, 0));
      if constexpr (MODE == 2)
        pmask[t] = __builtin_amdgcn_raw_buffer_load_b8(rmask, off == kSOOB ? kSOOB : off / 16, 0, 0);
      if constexpr (BNB && K3 == 0)
        bxp[t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rbx, off, 0, 0));
      if constexpr (BMK == 1)
        bmp[t] = __builtin_amdgcn_raw_buffer_load_b8(rbm, off == kSOOB ? kSOOB : off / 16, 0, 0);
      if constexpr (DUAL)
        bpp[t] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rbp, off, 0, 0));
    }
  };

  // chunk c's per-channel sums (8 waves' partials, fixed order) -> slab row blockIdx.x; DUAL: sum dz
  // is shared, the shortcut BN's sum dz x-hat_p is quantity 2
  auto write_slab = [&](int c) {
    const int which = tid >> 6, col = tid & 63;
    const float* sr = sred + (c & 1) * 8 * NQ * kSBN;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) t += sr[(w * NQ + which) * kSBN + col];
    const long o = (long)blockIdx.x * 2 * g.N + c * kSBN + col;
    if (which < 2) g.stats[o + (long)which * g.N] = t;
    if constexpr (DUAL) {
      if (which == 0) g.statsp[o] = t;
      if (which == 2) g.statsp[o + g.N] = t;
    }
  };
  issue(0);
  issue(1);
  constexpr int Y = PRE ? 2 * KS : 0;          // PRE: 16-B stores of the normalised A rows
  if constexpr (PRE) {
    // BN + ReLU of the A rows in registers (the loads above and the first chunks' DMAs are in
    // flight; the scale / shift reads wait for the A rows, in issue order), stored once as the
    // weight gradient's operand
    const __amdgpu_buffer_rsrc_t ry =
        srsrc(g.pre_y + m0 * g.lda, (uint32_t)(((long)(rows_blk - 1) * g.lda + K) * 2));
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k0 = ks * 32 + fq * 8;
      const float4 s0 = *reinterpret_cast<const float4*>(g.pre_sc + k0);
      const float4 s1 = *reinterpret_cast<const float4*>(g.pre_sc + k0 + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(g.pre_sh + k0);
      const float4 h1 = *reinterpret_cast<const float4*>(g.pre_sh + k0 + 4);
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float v[8];
        unpack8(__builtin_bit_cast(uint4, af[i][ks]), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(__builtin_fmaf(v[e], sc[e], sh[e]), 0.f);
        const uint4 pk = pack8(v);
        af[i][ks] = __builtin_bit_cast(bf16x8_t, pk);
        const int r = wave * kSWR + i * 16 + frow;
        const uint32_t off = r < rows_blk ? (uint32_t)((r * g.lda + k0) * 2) : kSOOB;
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) int, pk), ry, off, 0, 0);
      }
    }
  }
  prefetch(0);
  bf16_t* ws = stg + wave * kSWR * kSP;
  for (int c = 0; c < nch; ++c) {
    // this wave's DMAs of chunk c landed (everything issued after them may still fly) ...
    if (c >= 2) wait_vmc<2 * SST + 2 * L + D>();
    else if (c == 1) wait_vmc<2 * L + D + SST + Y>();
    else wait_vmc<D + L + Y>();
    if constexpr (HASPRM) {
      if (c == 0 && tid * 4 < g.N) {
#pragma unroll
        for (int a = 0; a < NPRM; ++a) *reinterpret_cast<float4*>(bprm + a * g.N + tid * 4) = prm[a];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(PROBE & 4)) raw_barrier();   // ... every wave's; every wave finished reading chunk c - 1's slot
    if (do_stats && c > 0 && tid < NQ * kSBN) write_slab(c - 1);
    issue(c + 2);
    const bf16_t* sb = lds + (c % 3) * CH;
    f32x4_t acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8_t bf[4];
      const int kp = ks >> 1, ch = (ks & 1) * 4 + fq;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = j * 16 + frow;
        bf[j] = *reinterpret_cast<const bf16x8_t*>(sb + kp * 64 * 64 + r * 64 + sswz(r, ch) * 8);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if constexpr (PROBE & 1) asm volatile("" ::"v"(bf[j]), "v"(af[i][ks]));
          else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    // stage the wave's 32 x 64 bf16 outputs (+ BN statistics from the rounded values)
    float s1[4], s2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s1[j] = s2[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fq * 4 + r;
          const bf16_t h = f2bf(acc[i][j][r]);
          if constexpr ((PROBE & 2) || NOST) asm volatile("" ::"v"(h));
          else ws[row * kSP + j * 16 + frow] = h;
          if (STATS && wave * kSWR + row < rows_blk) {
            const float q = bf2f(h);
            s1[j] += q;
            s2[j] += q * q;
          }
        }
    if constexpr (STATS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s1[j] += __shfl_xor(s1[j], 16, 64);
        s1[j] += __shfl_xor(s1[j], 32, 64);
        s2[j] += __shfl_xor(s2[j], 16, 64);
        s2[j] += __shfl_xor(s2[j], 32, 64);
      }
      if (fq == 0) {
        float* sr = sred + (c & 1) * 8 * NQ * kSBN + wave * NQ * kSBN;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sr[j * 16 + frow] = s1[j];
          sr[kSBN + j * 16 + frow] = s2[j];
        }
      }
    }
    // the staged tile is read back by other lanes of this wave: keep the reads behind the
    // writes (one wave's LDS instructions execute in order)
    asm volatile("" ::: "memory");
    if constexpr (NOST) {
      prefetch(c + 1);
      continue;                               // statistics only: nothing is stored
    }
    uint4 cv[S];
#pragma unroll
    for (int t = 0; t < S; ++t)
      cv[t] = (PROBE & 2) ? make_uint4(0u, 0u, 0u, (uint32_t)t)
                          : *reinterpret_cast<const uint4*>(ws + (t * 8 + er) * kSP + ec * 8);
    if constexpr (K3 > 0) {
      // RC: x = bf16(y2 . w3^T) for this chunk's 64 columns (the producing GEMM's chain: the same
      // fragments, k in order), staged over the C tile (already in cv) and read back per lane
      asm volatile("" ::: "memory");
      const bf16_t* sw3 = sb + CHB;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4_t a3[2] = {(f32x4_t){0.f, 0.f, 0.f, 0.f}, (f32x4_t){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < KS3; ++ks) {
          const int kp = ks >> 1, ch = (ks & 1) * 4 + fq;
          const int r = j * 16 + frow;
          const bf16x8_t wfr = *reinterpret_cast<const bf16x8_t*>(sw3 + kp * 64 * 64 + r * 64 + sswz(r, ch) * 8);
#pragma unroll
          for (int i = 0; i < 2; ++i)
            a3[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(yf[i][ks], wfr, a3[i], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ws[(i * 16 + fq * 4 + r) * kSP + j * 16 + frow] = f2bf(a3[i][r]);
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int t = 0; t < S; ++t)
        bxp[t] = *reinterpret_cast<const uint4*>(ws + (t * 8 + er) * kSP + ec * 8);
    }
    if constexpr (L != 0) wait_vmc<D>();      // this chunk's prefetched epilogue operands
    float b1[8], b2[8], b3[8], bmu[8], bis[8], bsc[8], bsh[8];
    if constexpr (BNB) {
#pragma unroll
      for (int e = 0; e < 8; ++e) b1[e] = b2[e] = b3[e] = 0.f;
      const int ch0 = c * kSBN + ec * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bmu[e] = bprm[ch0 + e];
        bis[e] = bprm[g.N + ch0 + e];
        // BMK 2: forward scale / shift; DUAL: the shortcut BN's mean / invstd
        if constexpr (BMK == 2 || DUAL) { bsc[e] = bprm[2 * g.N + ch0 + e]; bsh[e] = bprm[3 * g.N + ch0 + e]; }
      }
    }
    float asv[8], ahv[8];
    if constexpr (MODE == 3) {
      const int ch0 = c * kSBN + ec * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        asv[e] = bprm[ch0 + e];
        ahv[e] = bprm[g.N + ch0 + e];
      }
    }
#pragma unroll
    for (int t = 0; t < S; ++t) {
      uint4 v = cv[t];
      if constexpr (MODE == 3) {
        // the residual BatchNorm's apply, bit-identical to bn_apply_kernel (x * sc + sh, + res,
        // ReLU; the mask from the rounded output)
        float xv[8], rv[8], o[8];
        unpack8(v, xv);
        unpack8(pre[t], rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[e] = __builtin_fmaf(xv[e], asv[e], ahv[e]);
          o[e] += rv[e];
          o[e] = fmaxf(o[e], 0.f);
        }
        v = pack8(o);
        float ov[8];
        unpack8(v, ov);
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) bits |= (ov[e] > 0.f ? 1u : 0u) << e;
        const uint32_t mo = eoff(t, c);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)bits, ramask, mo == kSOOB ? kSOOB : mo / 16, 0, 0);
      } else if constexpr (MODE != 0) {
        float a[8], b[8];
        unpack8(v, a);
        unpack8(pre[t], b);
        if constexpr (MODE == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] += b[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] += (pmask[t] >> e) & 1u ? b[e] : 0.f;
        }
        v = pack8(a);
      }
      if constexpr (BNB) {
        if (wave * kSWR + t * 8 + er < rows_blk) {
          // the BatchNorm backward's reduce, on the gradient exactly as it is stored
          float gd[8], xv[8], pv[8];
          unpack8(v, gd);
          unpack8(bxp[t], xv);
          if constexpr (DUAL) unpack8(bpp[t], pv);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float dz = gd[e];
            if constexpr (BMK == 1) dz = (bmp[t] >> e) & 1u ? dz : 0.f;
            if constexpr (BMK == 2 && !DUAL) dz = __builtin_fmaf(xv[e], bsc[e], bsh[e]) > 0.f ? dz : 0.f;
            b1[e] += dz;
            b2[e] += dz * (xv[e] - bmu[e]) * bis[e];
            if constexpr (DUAL) b3[e] += dz * (pv[e] - bsc[e]) * bsh[e];
          }
        }
      }
      const uint32_t off = (PROBE & 8) ? kSOOB : eoff(t, c);
      const auto w = __builtin_bit_cast(__attribute__((ext_vector_type(4))) int, v);
      if (g.nt) __builtin_amdgcn_raw_buffer_store_b128(w, rc, off, 0, 2);   // nt
      else __builtin_amdgcn_raw_buffer_store_b128(w, rc, off, 0, 0);
    }
    asm volatile("" ::: "memory");            // next chunk's staging writes stay behind these reads
    if constexpr (BNB) {
      // the 8 row lanes sharing a column chunk (lanes ec, ec + 8, ..., ec + 56) meet by
      // cross-lane adds; lanes 0-7 hold the wave's sums of columns 8 ec .. 8 ec + 7
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        b1[e] += __shfl_xor(b1[e], 8, 64);
        b1[e] += __shfl_xor(b1[e], 16, 64);
        b1[e] += __shfl_xor(b1[e], 32, 64);
        b2[e] += __shfl_xor(b2[e], 8, 64);
        b2[e] += __shfl_xor(b2[e], 16, 64);
        b2[e] += __shfl_xor(b2[e], 32, 64);
        if constexpr (DUAL) {
          b3[e] += __shfl_xor(b3[e], 8, 64);
          b3[e] += __shfl_xor(b3[e], 16, 64);
          b3[e] += __shfl_xor(b3[e], 32, 64);
        }
      }
      if (er == 0) {
        float* sr = sred + (c & 1) * 8 * NQ * kSBN + wave * NQ * kSBN + ec * 8;
        *reinterpret_cast<float4*>(sr) = make_float4(b1[0], b1[1], b1[2], b1[3]);
        *reinterpret_cast<float4*>(sr + 4) = make_float4(b1[4], b1[5], b1[6], b1[7]);
        *reinterpret_cast<float4*>(sr + kSBN) = make_float4(b2[0], b2[1], b2[2], b2[3]);
        *reinterpret_cast<float4*>(sr + kSBN + 4) = make_float4(b2[4], b2[5], b2[6], b2[7]);
        if constexpr (DUAL) {
          *reinterpret_cast<float4*>(sr + 2 * kSBN) = make_float4(b3[0], b3[1], b3[2], b3[3]);
          *reinterpret_cast<float4*>(sr + 2 * kSBN + 4) = make_float4(b3[4], b3[5], b3[6], b3[7]);
        }
      }
    }
    prefetch(c + 1);
  }
  DTF_WAIT_VM(0);       // the trailing out-of-range DMAs still target the ring
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  if (do_stats && tid < NQ * kSBN) write_slab(nch - 1);
}

template <int K, int MODE, bool STATS, int BMK = -1, bool PRE = false, int PROBE = 0,
          bool DUAL = false, bool NOST = false, int K3 = 0>
void launch_stream(const StreamArgs& g, hipStream_t st) {
  constexpr size_t BASE = (size_t)3 * kSBN * (K + K3) * 2 + (size_t)8 * kSWR * kSP * 2 +
                          (size_t)2 * 8 * (DUAL ? 3 : 2) * kSBN * 4;
  static_assert(BASE <= 160 * 1024, "gemm_stream LDS");
  // BNB / APPLY: + the per-channel parameter arrays
  const size_t LDS = BASE + (BMK >= 0 ? (size_t)((BMK == 2 || DUAL) ? 4 : 2) * g.N * 4
                             : MODE == 3 ? (size_t)2 * g.N * 4 : 0);
  if (LDS > 160 * 1024) throw std::runtime_error("gemm_stream: per-channel parameters exceed LDS");
  auto kern = gemm_stream_kernel<K, MODE, STATS, BMK, PRE, PROBE, DUAL, NOST, K3>;
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024));
    attr = true;
  }
  const unsigned blocks = (unsigned)((g.M + kSBM - 1) / kSBM);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kST), LDS, st, g);
}

// timing probe of the kind-1 BN-backward epilogue (PROBE bits 4 / 8 above; wrong results): only
// in a probe build (-DDTF_PROBES, tools only)
#ifdef DTF_PROBES
static int g_stream_bnb_probe = 0;
#endif

template <int K, int MODE>
void launch_stream_bnb(const StreamArgs& g, int bmk, hipStream_t st) {
  if (g.y2) {            // RC: the residual BN's input recomputed (kind 1, K <= 128, K3 64 / 128)
    if constexpr (K <= 128) {
      if (bmk != 1 || g.bxp) throw std::runtime_error("gemm_stream_bnb: RC needs kind 1, no dual");
      if (g.k3 == 64) launch_stream<K, MODE, false, 1, false, 0, false, false, 64>(g, st);
      else if (g.k3 == 128) launch_stream<K, MODE, false, 1, false, 0, false, false, 128>(g, st);
      else throw std::runtime_error("gemm_stream_bnb: RC depth K3 in {64, 128}");
      return;
    }
    throw std::runtime_error("gemm_stream_bnb: RC needs K <= 128");
  }
  if (g.bxp) launch_stream<K, MODE, false, 1, false, 0, true>(g, st);
  else if (bmk == 1) {
#ifdef DTF_PROBES
    switch (g_stream_bnb_probe) {
      case 4: launch_stream<K, MODE, false, 1, false, 4>(g, st); break;
      case 8: launch_stream<K, MODE, false, 1, false, 8>(g, st); break;
      case 12: launch_stream<K, MODE, false, 1, false, 12>(g, st); break;
      default: launch_stream<K, MODE, false, 1>(g, st); break;
    }
#else
    launch_stream<K, MODE, false, 1>(g, st);
#endif
  }
  else if (bmk == 2) launch_stream<K, MODE, false, 2>(g, st);
  else launch_stream<K, MODE, false, 0>(g, st);
}

template <int K>
void launch_stream_k(const StreamArgs& g, int bmk, hipStream_t st) {
  if (g.pre_y) {
    if (g.nost) {
      if (!g.stats) throw std::runtime_error("gemm_stream_pre: no-store form needs statistics");
      launch_stream<K, 0, true, -1, true, 0, false, true>(g, st);
    } else if (g.stats) launch_stream<K, 0, true, -1, true>(g, st);
    else launch_stream<K, 0, false, -1, true>(g, st);
  } else if (g.asc) {
    launch_stream<K, 3, false>(g, st);
  } else if (g.bx || g.y2) {
    if (g.Cin) launch_stream_bnb<K, 1>(g, bmk, st);
    else if (g.acc_mask) launch_stream_bnb<K, 2>(g, bmk, st);
    else launch_stream_bnb<K, 0>(g, bmk, st);
  } else if (g.stats) launch_stream<K, 0, true>(g, st);
  else if (g.Cin) launch_stream<K, 1, false>(g, st);
  else if (g.acc_mask) launch_stream<K, 2, false>(g, st);
  else launch_stream<K, 0, false>(g, st);
}

}  // namespace

// true if the row-streaming kernel takes this GEMM (see the header); statistics slab rows are
// ceil(M / 256), the same as dtf_gemm_tile_rows
bool dtf_gemm_stream_ok(int M, int N, int K, int lda, int ldb, int ldc) {
  return (K == 64 || K == 128 || K == 256) && N % kSBN == 0 && N >= kSBN && M > 0 &&
         lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 && lda >= K && ldb >= K && ldc >= N &&
         (long)kSBM * lda * 2 < (1L << 31) && (long)kSBM * ldc * 2 < (1L << 31) &&
         (long)N * ldb * 2 < (1L << 31);
}

static void run_stream(StreamArgs& g, int K, int bmk, hipStream_t st) {
  switch (K) {
    case 64: launch_stream_k<64>(g, bmk, st); break;
    case 128: launch_stream_k<128>(g, bmk, st); break;
    default: launch_stream_k<256>(g, bmk, st); break;
  }
}

void dtf_gemm_stream(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int lda,
                     int ldb, int ldc, const bf16_t* Cin, float* stats, const bf16_t* acc_src,
                     const uint8_t* acc_mask, int nt, hipStream_t st) {
  if (!dtf_gemm_stream_ok(M, N, K, lda, ldb, ldc))
    throw std::runtime_error("gemm_stream: K in {64,128,256}, N % 64 == 0, aligned strides");
  if ((stats != nullptr) + (Cin != nullptr) + (acc_mask != nullptr) > 1)
    throw std::runtime_error("gemm_stream: one epilogue mode (stats | Cin | masked acc)");
  if (acc_mask && (!acc_src || ldc != N))
    throw std::runtime_error("gemm_stream: masked accumulation needs acc_src and a dense C");
  StreamArgs g{A, B, C, Cin, acc_src, acc_mask, stats, M, N, lda, ldb, ldc, nt};
  run_stream(g, K, -1, st);
}

// A data-gradient GEMM (plain, Cin or masked accumulate) that also emits the BN-backward sums
// of the BatchNorm whose output gradient C is: part [ceil(M/256)][2][N] (sum dz, sum dz x-hat).
// kind: 0 no ReLU, 1 ReLU bit mask `bmask`, 2 ReLU recomputed from x with (bsc, bsh).
void dtf_gemm_stream_bnb(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K,
                         int lda, int ldb, int ldc, const bf16_t* Cin, const bf16_t* acc_src,
                         const uint8_t* acc_mask, const bf16_t* bx, const float* bmean,
                         const float* binv, const float* bsc, const float* bsh,
                         const uint8_t* bmask, int kind, float* part, int nt, hipStream_t st,
                         const bf16_t* y2, const bf16_t* w3, int k3) {
  if (!dtf_gemm_stream_ok(M, N, K, lda, ldb, ldc) || ldc != N || N > 2048)
    throw std::runtime_error("gemm_stream_bnb: stream shape, dense C, N <= 2048");
  if (Cin && acc_mask) throw std::runtime_error("gemm_stream_bnb: Cin or masked acc, not both");
  if (acc_mask && !acc_src) throw std::runtime_error("gemm_stream_bnb: masked acc needs acc_src");
  const bool rc = y2 != nullptr;
  if ((!bx && !rc) || !bmean || !binv || !part || kind < 0 || kind > 2 || (kind == 1 && !bmask) ||
      (kind == 2 && !(bsc && bsh)) || (rc && (!w3 || (k3 != 64 && k3 != 128) || kind != 1)))
    throw std::runtime_error("gemm_stream_bnb: BatchNorm operands");
  StreamArgs g{A, B, C, Cin, acc_src, acc_mask, part, M, N, lda, ldb, ldc, nt,
               bx, bmean, binv, bsc, bsh, bmask};
  g.y2 = y2;
  g.w3 = w3;
  g.k3 = rc ? k3 : 0;
  run_stream(g, K, kind, st);
}

// dtf_gemm_stream_bnb for the output gradient of relu(BN(x) + BN_p(xp)) (kind 1, bit mask): also
// the shortcut BN's sums (sum dz, sum dz xp-hat) into part_p.  Replaces the dual reduce pass.
void dtf_gemm_stream_bnb_dual(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K,
                              int lda, int ldb, int ldc, const bf16_t* Cin, const bf16_t* acc_src,
                              const uint8_t* acc_mask, const bf16_t* bx, const float* bmean,
                              const float* binv, const uint8_t* bmask, float* part,
                              const bf16_t* bxp, const float* bmeanp, const float* binvp,
                              float* part_p, hipStream_t st) {
  if (!dtf_gemm_stream_ok(M, N, K, lda, ldb, ldc) || ldc != N || N > 2048)
    throw std::runtime_error("gemm_stream_bnb_dual: stream shape, dense C, N <= 2048");
  if (Cin && acc_mask) throw std::runtime_error("gemm_stream_bnb_dual: Cin or masked acc, not both");
  if (acc_mask && !acc_src) throw std::runtime_error("gemm_stream_bnb_dual: masked acc needs acc_src");
  if (!bx || !bmean || !binv || !bmask || !part || !bxp || !bmeanp || !binvp || !part_p)
    throw std::runtime_error("gemm_stream_bnb_dual: BatchNorm operands");
  StreamArgs g{A, B, C, Cin, acc_src, acc_mask, part, M, N, lda, ldb, ldc, 0,
               bx, bmean, binv, nullptr, nullptr, bmask};
  g.bxp = bxp;
  g.bmeanp = bmeanp;
  g.binvp = binvp;
  g.statsp = part_p;
  run_stream(g, K, 1, st);
}

// C = relu(BN(X)) . B^T with the BatchNorm + ReLU applied to the A rows in registers (scale /
// shift per reduction channel, the BN apply pass's arithmetic) and the normalised rows written
// to y (same layout as X) for the weight gradient; optional BN statistics of C.  The BN apply
// pass over X and the GEMM's re-read of its output become one read of X.
void dtf_gemm_stream_pre(const bf16_t* X, const bf16_t* B, bf16_t* C, int M, int N, int K,
                         const float* pre_sc, const float* pre_sh, bf16_t* y, float* stats,
                         hipStream_t st, int nostore) {
  if (!dtf_gemm_stream_ok(M, N, K, K, K, N) || !pre_sc || !pre_sh || !y)
    throw std::runtime_error("gemm_stream_pre: stream shape and BatchNorm operands");
  if (nostore && !stats) throw std::runtime_error("gemm_stream_pre: no-store form needs stats");
  StreamArgs g{X, B, C, nullptr, nullptr, nullptr, stats, M, N, K, K, N, 0};
  g.pre_sc = pre_sc;
  g.pre_sh = pre_sh;
  g.pre_y = y;
  g.nost = nostore ? 1 : 0;
  run_stream(g, K, -1, st);
}

// The residual BatchNorm's apply on a conv output that was never stored (lazy x3): Y = relu(
// bf16(A . W^T) * sc + sh + res) and its ReLU bit mask, with A = the conv's input [M][K] and the
// GEMM the producing stream GEMM's exact chain -- bit-identical to storing the conv output and
// running the apply pass over it.
void dtf_gemm_stream_apply(const bf16_t* A, const bf16_t* W, bf16_t* Y, int M, int N, int K,
                           const bf16_t* res, const float* sc, const float* sh, uint8_t* mask,
                           hipStream_t st) {
  if (!dtf_gemm_stream_ok(M, N, K, K, K, N) || !res || !sc || !sh || !mask || N > 4096)
    throw std::runtime_error("gemm_stream_apply: stream shape and BatchNorm operands");
  StreamArgs g{A, W, Y, res, nullptr, nullptr, nullptr, M, N, K, K, N, 0};
  g.asc = sc;
  g.ash = sh;
  g.amask = mask;
  run_stream(g, K, -1, st);
}

#ifdef DTF_PROBES
void dtf_gemm_stream_set_bnb_probe(int v) { g_stream_bnb_probe = v; }
#else
void dtf_gemm_stream_set_bnb_probe(int v) {
  if (v) throw std::runtime_error("gemm_stream_set_bnb_probe: a timing probe with wrong results; "
                                  "build with DTF_HIP_EXTRA_FLAGS=-DDTF_PROBES (tools only)");
}
#endif

// timing probes of the plain K = 256 kernel (see PROBE above)
void dtf_gemm_stream_probe(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int probe,
                           hipStream_t st) {
#ifndef DTF_PROBES
  (void)A; (void)B; (void)C; (void)M; (void)N; (void)probe; (void)st;
  throw std::runtime_error("gemm_stream_probe: timing probes need a DTF_PROBES build (tools only)");
#else
  if (!dtf_gemm_stream_ok(M, N, 256, 256, 256, N)) throw std::runtime_error("stream probe shape");
  StreamArgs g{A, B, C, nullptr, nullptr, nullptr, nullptr, M, N, 256, 256, N, 0};
  switch (probe) {
    case 1: launch_stream<256, 0, false, -1, false, 1>(g, st); break;
    case 2: launch_stream<256, 0, false, -1, false, 2>(g, st); break;
    case 4: launch_stream<256, 0, false, -1, false, 4>(g, st); break;
    case 8: launch_stream<256, 0, false, -1, false, 8>(g, st); break;
    case 10: launch_stream<256, 0, false, -1, false, 10>(g, st); break;
    case 11: launch_stream<256, 0, false, -1, false, 11>(g, st); break;
    case 15: launch_stream<256, 0, false, -1, false, 15>(g, st); break;
    default: launch_stream<256, 0, false, -1, false, 0>(g, st); break;
  }
#endif
}
