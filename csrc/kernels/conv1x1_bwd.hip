// Fused backward of ResNet-50's first-stage expanding 1x1 conv (c3: 64 -> 256 channels) whose
// input is relu(BN(x)) (ops/native.py _BnReluConv1x1):
//
//   dY[m, c]   = sum_k dO[m, k] W[k, c]                  (data gradient, bf16 out)
//   dW[k, c]  += sum_m dO[m, k] Y[m, c]                  (weight gradient, fp32 slab per block)
//   BN sums[c] = sum_m dz, sum_m dz (x - mean) invstd,   dz = dY * [x sc + sh > 0]
//
// Unfused these are three passes -- the weight-gradient kernel (reads dO, Y), the data-gradient
// GEMM (reads dO, writes dY) and the BN backward's reduce (reads dY, x): 1536 B of HBM traffic per
// row.  Here ONE pass reads dO, Y and x and writes dY: 896 B per row; the 2 x 2 x 64 x 256 FLOPs
// per row are ~5% of what the MFMA pipes could do in the time the bytes take, so the kernel is
// purely a streaming problem.  (profiles/measurements/r3_conv_roofline_b1984.jsonl: the dgrad and
// wgrad passes of this layer alone take 0.75 ms each at batch 1984.)
//
// Design (persistent: one block of 8 waves per CU, 64-row tiles walked with a grid stride):
//   * dO (64 x 256), Y (64 x 64) and x (64 x 64) tiles stream through a 3-slot LDS ring by
//     LDS-DMA, two tiles ahead, with source-side XOR swizzles chosen for the reads below;
//   * data gradient with the operands swapped -- A = W^T rows (this wave's 16 channels, whole K,
//     held in 32 VGPRs for the kernel's lifetime), B = dO rows from LDS -- so every lane ends up
//     with 4 CONSECUTIVE channels of one row: one 8-byte store of dY, one 8-byte LDS read of x
//     for the BN sums (computed on dY exactly as it is stored, like gemm_stream.hip's epilogue);
//   * weight gradient: the wave owns dW rows 32 w .. 32 w + 31 x all 64 channels (8 MFMA
//     accumulators, 32 fp32 per lane) for ALL of the block's tiles; both operands are read with
//     the hardware transpose read ds_read_b64_tr_b16 (the reduction runs over tile rows);
//   * at the end every block writes one fp32 dW slab [256][64] and one BN slab row [2][64]; the
//     host reduces the slabs in fixed order (deterministic; slab_reduce / bn_bwd_finalize_g).
// Only global memory traffic per tile per wave: 6 DMA instructions + 2 dY stores, so the counted
// vmcnt waits at the top of a tile are exact (see `top`).
#include <stdexcept>
#include <string>

#include "common.h"

namespace {

constexpr int kT = 512;              // threads: 8 waves
constexpr int kTM = 64;              // rows per tile
constexpr int kC = 64;               // conv input channels (dY / Y / x width)
constexpr int kK = 256;              // conv output channels (dO width)
constexpr int kNB = 3;               // ring slots
constexpr int kDO = kTM * kK;        // bf16 per dO tile (32 KB)
constexpr int kYT = kTM * kC;        // bf16 per Y / x tile (8 KB)
constexpr int kSlot = kDO + 2 * kYT; // bf16 per ring slot (48 KB)
constexpr size_t kLds = (size_t)kNB * kSlot * 2 + 2 * 2 * kC * 4;   // + BN partials [2][2][64]
static_assert(kLds <= 160 * 1024, "conv1x1_bwd LDS");

typedef __attribute__((ext_vector_type(4))) short s4_t;
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

// 16-B chunk swizzles (physical chunk = logical chunk ^ swz(row)):
//  dO, 512-B rows: the 16 rows of a dgrad B-fragment read (ds_read_b128, 16 lanes / pass) hit 16
//    different 16-B bank slots; the 8 rows of a transpose-read half-wave keep their 32-B column
//    pair adjacent and land on 8 different pairs
DTF_DEV int swz_o(int r) { return 2 * (r & 7) + ((r >> 3) & 1); }
//  Y, 128-B rows (transpose reads only): 8 rows x one 32-B pair -> 16 distinct slots
DTF_DEV int swz_y(int r) { return 2 * ((r >> 1) & 3); }
//  x, 128-B rows (8-B reads of 16 rows x one chunk per half-wave)
DTF_DEV int swz_x(int r) { return (r >> 1) & 7; }

template <int RP>
DTF_DEV int sidx(int r, int c, int s) { return r * RP + (((c >> 3) ^ s) << 3) + (c & 7); }

// 8 reduction rows x one column as an MFMA operand (key permutation: j < 4 -> row0 + 4g + j,
// j >= 4 -> row0 + 16 + 4g + j - 4; the same in both operands of a product)
template <int RP, int W>
DTF_DEV bf16x8_t tr8(const bf16_t* base, int row0, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int r = row0 + 4 * g + (i >> 2), c = col0 + 4 * (i & 3);
  const int s0 = W == 0 ? swz_o(r) : swz_y(r);
  const int s1 = W == 0 ? swz_o(r + 16) : swz_y(r + 16);
  const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(base + sidx<RP>(r, c, s0)));
  const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(base + sidx<RP>(r + 16, c, s1)));
  return (bf16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

DTF_DEV f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int N>
DTF_DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct C1Args {
  const bf16_t* dout;   // [M][256]  gradient of the conv output
  const bf16_t* wt;     // [64][256] W^T (wt[c][k] = W[k][c])
  const bf16_t* y;      // [M][64]   the conv input relu(BN(x))
  const bf16_t* x;      // [M][64]   the BatchNorm input
  const float* mean;
  const float* inv;
  const float* sc;      // forward scale / shift (ReLU recomputed from x)
  const float* sh;
  bf16_t* dy;           // [M][64]   data gradient (of y)
  float* wpart;         // [grid][256][64]
  float* bpart;         // [grid][2][64]
  int M;
};

__global__ void __launch_bounds__(kT, 1) conv1x1_bwd_kernel(const C1Args g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  float* sred = reinterpret_cast<float*>(lds + kNB * kSlot);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, gq = lane >> 4;
  const int ntiles = g.M / kTM;
  const int nmy = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int cb = wave & 3, mh = wave >> 2;     // data gradient: channels 16 cb.., rows 32 mh..
  const int c0 = cb * 16 + 4 * gq;             // this lane's 4 output channels

  // W^T fragments: this wave's 16 channels x the whole reduction (loaded once)
  bf16x8_t wf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    wf[ks] = *reinterpret_cast<const bf16x8_t*>(g.wt + (cb * 16 + li) * kK + ks * 32 + gq * 8);
  const float4 pmu = *reinterpret_cast<const float4*>(g.mean + c0);
  const float4 pin = *reinterpret_cast<const float4*>(g.inv + c0);
  const float4 psc = *reinterpret_cast<const float4*>(g.sc + c0);
  const float4 psh = *reinterpret_cast<const float4*>(g.sh + c0);
  const float mu[4] = {pmu.x, pmu.y, pmu.z, pmu.w}, is[4] = {pin.x, pin.y, pin.z, pin.w};
  const float sc[4] = {psc.x, psc.y, psc.z, psc.w}, sh[4] = {psh.x, psh.y, psh.z, psh.w};

  const uint32_t lds0 = lds_addr(lds);
  // tile i of this block -> slot i % 3: dO rows 2q, 2q + 1 per instruction (q = wave + 8 j),
  // Y / x rows 8 wave .. 8 wave + 7
  auto issue = [&](int i) {
    const long m0 = ((long)blockIdx.x + (long)i * gridDim.x) * kTM;
    const i32x4_t ro = rsrc_quad(g.dout + m0 * kK, (uint32_t)(kDO * 2));
    const i32x4_t ry = rsrc_quad(g.y + m0 * kC, (uint32_t)(kYT * 2));
    const i32x4_t rx = rsrc_quad(g.x + m0 * kC, (uint32_t)(kYT * 2));
    const uint32_t base = lds0 + (uint32_t)((i % kNB) * kSlot * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = wave + 8 * j, r = 2 * q + (lane >> 5), s = lane & 31;
      dma16(ro, base + (uint32_t)q * 1024u, (uint32_t)((r * kK + ((s ^ swz_o(r)) << 3)) * 2));
    }
    const int r = 8 * wave + (lane >> 3), s = lane & 7;
    dma16(ry, base + (uint32_t)(kDO * 2 + wave * 1024), (uint32_t)((r * kC + ((s ^ swz_y(r)) << 3)) * 2));
    dma16(rx, base + (uint32_t)((kDO + kYT) * 2 + wave * 1024),
          (uint32_t)((r * kC + ((s ^ swz_x(r)) << 3)) * 2));
  };

  f32x4_t aw[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) aw[a][b] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (nmy > 1) issue(1);
  for (int i = 0; i < nmy; ++i) {
    // top: this wave's DMAs of tile i landed.  Younger vector-memory ops at this point: tile
    // i + 1's DMAs (6, if it exists) and the dY stores of tiles i - 1 and i - 2 (2 each).
    const bool more = i + 1 < nmy;
    if (i == 0) { if (more) wait_vm<6>(); else wait_vm<0>(); }
    else if (i == 1) { if (more) wait_vm<8>(); else wait_vm<2>(); }
    else { if (more) wait_vm<10>(); else wait_vm<4>(); }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();                  // every wave's DMAs landed; slot (i + 2) % 3 was read in i - 1
    if (i + 2 < nmy) issue(i + 2);
    const bf16_t* sO = lds + (i % kNB) * kSlot;
    const bf16_t* sY = sO + kDO;
    const bf16_t* sX = sY + kYT;

    // data gradient: rows 32 mh + 16 f + li, channels c0 .. c0 + 3 (after the MFMA's transpose)
    f32x4_t ad[2] = {(f32x4_t){0.f, 0.f, 0.f, 0.f}, (f32x4_t){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int m = mh * 32 + f * 16 + li;
        const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(sO + sidx<kK>(m, ks * 32 + gq * 8, swz_o(m)));
        ad[f] = mfma16(wf[ks], b, ad[f]);
      }
    }
    // weight gradient: dW rows 32 wave + 16 kb + .., channels 16 cb2 + .., over the tile's rows
#pragma unroll
    for (int ms = 0; ms < 2; ++ms) {
      bf16x8_t fa[2], fb[4];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) fa[kb] = tr8<kK, 0>(sO, 32 * ms, wave * 32 + kb * 16, lane);
#pragma unroll
      for (int cb2 = 0; cb2 < 4; ++cb2) fb[cb2] = tr8<kC, 1>(sY, 32 * ms, cb2 * 16, lane);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int cb2 = 0; cb2 < 4; ++cb2) aw[kb][cb2] = mfma16(fa[kb], fb[cb2], aw[kb][cb2]);
    }
    // epilogue: dY (bf16) + the BatchNorm backward sums on the stored values
    const long m0 = ((long)blockIdx.x + (long)i * gridDim.x) * kTM;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int m = mh * 32 + f * 16 + li;
      const uint2 pk = make_uint2(pack2(ad[f][0], ad[f][1]), pack2(ad[f][2], ad[f][3]));
      *reinterpret_cast<uint2*>(g.dy + (m0 + m) * kC + c0) = pk;
      const uint2 xr = *reinterpret_cast<const uint2*>(sX + sidx<kC>(m, c0, swz_x(m)));
      const float gd[4] = {__builtin_bit_cast(float, pk.x << 16), __builtin_bit_cast(float, pk.x & 0xffff0000u),
                           __builtin_bit_cast(float, pk.y << 16), __builtin_bit_cast(float, pk.y & 0xffff0000u)};
      const float xv[4] = {__builtin_bit_cast(float, xr.x << 16), __builtin_bit_cast(float, xr.x & 0xffff0000u),
                           __builtin_bit_cast(float, xr.y << 16), __builtin_bit_cast(float, xr.y & 0xffff0000u)};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dz = __builtin_fmaf(xv[e], sc[e], sh[e]) > 0.f ? gd[e] : 0.f;
        s1[e] += dz;
        s2[e] += dz * (xv[e] - mu[e]) * is[e];
      }
    }
  }
  DTF_WAIT_VM(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();

  // BN partials: the 16 row lanes sharing a channel group meet by cross-lane adds, then the two
  // waves sharing cb in fixed order
#pragma unroll
  for (int e = 0; e < 4; ++e) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s1[e] += __shfl_xor(s1[e], o, 64);
      s2[e] += __shfl_xor(s2[e], o, 64);
    }
  }
  if (li == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sred[(mh * 2 + 0) * kC + c0 + e] = s1[e];
      sred[(mh * 2 + 1) * kC + c0 + e] = s2[e];
    }
  }
  __syncthreads();
  if (tid < 2 * kC) {
    const int which = tid >> 6, col = tid & 63;
    g.bpart[((long)blockIdx.x * 2 + which) * kC + col] =
        sred[which * kC + col] + sred[(2 + which) * kC + col];
  }
  // dW slab: lane holds dW[32 wave + 16 kb + 4 gq + r][16 cb2 + li]
  float* wp = g.wpart + (long)blockIdx.x * kK * kC;
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int cb2 = 0; cb2 < 4; ++cb2)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        wp[(wave * 32 + kb * 16 + 4 * gq + r) * kC + cb2 * 16 + li] = aw[kb][cb2][r];
}

int g_c1_grid = 0;   // 0 = one block per CU

int c1_blocks(int M) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int want = g_c1_grid > 0 ? g_c1_grid : cus;
  const int ntiles = M / kTM;
  return ntiles < want ? ntiles : want;
}

}  // namespace

bool dtf_conv1x1_bwd_ok(int M, int C, int K) { return C == kC && K == kK && M > 0 && M % kTM == 0; }

// number of slab rows (blocks) the fused backward writes for M rows
int dtf_conv1x1_bwd_blocks(int M) {
  if (M <= 0 || M % kTM) throw std::runtime_error("conv1x1_bwd: M % 64 != 0");
  return c1_blocks(M);
}

void dtf_conv1x1_bwd_set_grid(int n) { g_c1_grid = n; }

void dtf_conv1x1_bwd(const bf16_t* dout, const bf16_t* wt, const bf16_t* y, const bf16_t* x,
                     const float* mean, const float* inv, const float* sc, const float* sh,
                     bf16_t* dy, float* wpart, float* bpart, int M, hipStream_t st) {
  if (M <= 0 || M % kTM) throw std::runtime_error("conv1x1_bwd: M must be a positive multiple of 64");
  const void* ptrs[] = {dout, wt, y, x, mean, inv, sc, sh, dy, wpart, bpart};
  for (const void* p : ptrs)
    if (!p || (reinterpret_cast<uintptr_t>(p) & 15))
      throw std::runtime_error("conv1x1_bwd: null or misaligned operand");
  static bool attr = false;
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)conv1x1_bwd_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds));
    attr = true;
  }
  C1Args g{dout, wt, y, x, mean, inv, sc, sh, dy, wpart, bpart, M};
  hipLaunchKernelGGL(conv1x1_bwd_kernel, dim3(c1_blocks(M)), dim3(kT), kLds, st, g);
}
