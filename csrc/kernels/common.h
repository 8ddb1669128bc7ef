// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of distributedtensorflow_amd.
//
// Conventions
//  * bf16 tensors are carried as `uint16_t` storage; conversion goes through the clang
//    `__bf16` type so hipcc emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving) — see
//    MI355X_MICROARCH.md "Correctness boundaries".
//  * memory-bound kernels move 16 B per lane (8 x bf16 / 4 x f32) — guide Guideline 13.
//  * wave = 64 lanes; blocks are multiples of 64 threads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DTF_DEV __device__ __forceinline__

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // one MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) short bf16x4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

DTF_DEV float bf2f(bf16_t v) { return __builtin_bit_cast(float, ((uint32_t)v) << 16); }
DTF_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// 8 bf16 packed in a uint4 (16 bytes)
DTF_DEV void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __builtin_bit_cast(float, w[i] << 16);
    f[2 * i + 1] = __builtin_bit_cast(float, w[i] & 0xffff0000u);
  }
}
DTF_DEV uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
DTF_DEV uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2(f[0], f[1]);
  r.y = pack2(f[2], f[3]);
  r.z = pack2(f[4], f[5]);
  r.w = pack2(f[6], f[7]);
  return r;
}

// 16-B store, non-temporal when `nt` (a wave-uniform flag): outputs written once and read by a
// later kernel pass, far larger than L2 / MALL
typedef uint32_t u32x4_st __attribute__((ext_vector_type(4)));
DTF_DEV void st16(void* p, const uint4& v, bool nt) {
  if (nt) {
    const u32x4_st w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4_st*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}

DTF_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DTF_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline int dtf_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// XCD-aware bijective remap of a 1-D block id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks that share an XCD (b % 8) get a contiguous range of logical ids, so
// neighbouring output tiles (which share operand panels) hit the same L2.  Speed only.
DTF_DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// ---- LDS-DMA (buffer_load_dwordx4 ... lds) helpers shared by the MFMA conv kernels
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((ext_vector_type(4))) int i32x4_t;

// Buffer descriptor as a plain SGPR quad (for inline asm): base, stride 0, num_records = bytes.
DTF_DEV i32x4_t rsrc_quad(const void* p, uint32_t bytes) {
  const unsigned long long b = (unsigned long long)p;
  return (i32x4_t){__builtin_amdgcn_readfirstlane((int)(uint32_t)b),
                   __builtin_amdgcn_readfirstlane((int)((b >> 32) & 0xFFFFu)), (int)bytes,
                   0x00020000};
}
DTF_DEV uint32_t lds_addr(const bf16_t* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(const lds_void_t*)p);
}
// One 1-KB LDS-DMA wave-instruction: lane l's 16 bytes at `voff` land at LDS byte lds + 16 l.
// Issued as inline asm on purpose: the compiler then does not treat it as an LDS store and does
// not insert its own (over-conservative) vmcnt waits in front of the fragment reads -- the
// kernel waits with explicit counted vmcnt instead.  M0 is saved and restored around it.
DTF_DEV void dma16(const i32x4_t& r, uint32_t lds, uint32_t voff) {
  uint32_t save;
  // the LDS base is wave-uniform by contract; readfirstlane states it where the compiler's
  // uniformity analysis lost track (a no-op when the value already lives in an SGPR)
  const uint32_t l = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tbuffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(save) : "s"(l), "v"(voff), "s"(r) : "memory");
}
#define DTF_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
DTF_DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- BatchNorm backward apply: dx = A dz + B x + C per channel, in ONE explicit operation order
// (every kernel that forms it -- the apply passes, the pool-fused stem pass, the fused 1x1
// backward that consumes it without storing -- must round identically)
DTF_DEV float bn_bwd_dx(float a, float dz, float b, float x, float c) {
  return __builtin_fmaf(a, dz, b * x) + c;
}

// 3x3 / 2 max-pool backward (pad 1) for the 2 x 2 block of input pixels (2a + ii, 2b + jj): the
// gradients of the <= 4 pooled outputs (a .. a + 1, b .. b + 1) whose argmax byte (window
// position r * 3 + s) names the pixel, rounded to bf16 as a stored d(pool input) would be.
// Shared by pool.hip (pool3s2_bn_bwd_kernel) and conv_wgrad.hip (the stem wgrad that forms its
// dY on load): both must produce the identical bits.
DTF_DEV void pool3s2_gather(const uint4 (&dyr)[4], const uint2 (&amr)[4], int a, int b, int P,
                            int Q, float (&g)[4][8]) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) g[k][e] = 0.f;
#pragma unroll
  for (int da = 0; da < 2; ++da) {
    if (a + da >= P) continue;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      if (b + db >= Q) continue;
      float gv[8];
      unpack8(dyr[da * 2 + db], gv);
      const uint32_t aw[2] = {amr[da * 2 + db].x, amr[da * 2 + db].y};
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int r = ii - 2 * da + 1, s = jj - 2 * db + 1;
          if (r < 0 || r > 2 || s < 0 || s > 2) continue;
          const uint32_t me = (uint32_t)(r * 3 + s);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (((aw[e >> 2] >> ((e & 3) * 8)) & 0xffu) == me) g[ii * 2 + jj][e] += gv[e];
        }
    }
  }
  // the unfused path stores d(BN output) as bf16: round exactly like it
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) g[k][e] = bf2f(f2bf(g[k][e]));
}

// ---- GELU (tanh approximation, BERT's "gelu") shared by the NLP kernels and the GEMM epilogue
constexpr float kGeluK0 = 0.7978845608028654f;   // sqrt(2/pi)
constexpr float kGeluK1 = 0.044715f;

// tanh on v_exp_f32 / v_rcp_f32 (libm tanhf is a long branchy sequence; the absolute error here
// is ~1e-7, far below the bf16 output rounding).
// tanh-GELU with u = K0 (x + K1 x^3) and r = 1 / (1 + e^{2u}): tanh u = 1 - 2 r, so
//   gelu(x)  = 0.5 x (1 + tanh u) = x - x r
//   gelu'(x) = (1 - r) (1 + x r (2 K0 + 6 K0 K1 x^2))      [1 - tanh^2 u = 4 r (1 - r)]
// -- 5 (forward) / 9 (derivative) plain VALU ops besides v_exp_f32 + v_rcp_f32, against 10 / 16
// for the tanh form: these run in the GEMM epilogues of BERT's FFN (gemm.hip EPI 8 / 16), where
// the GELU arithmetic measured ~50 us of a ~360 us call.  e^{2u} = inf -> r = 0 (gelu = x,
// gelu' = 1); e^{2u} = 0 -> r = 1 (gelu = 0, gelu' = 0), as the tanh form gives, for every
// finite x.  Non-finite x: gelu(+inf) is NaN here (the tanh form gave +inf; -inf is NaN in
// both) -- a non-finite pre-activation has already poisoned the step either way.
constexpr float kGeluE0 = 2.f * kGeluK0 * 1.4426950408889634f;   // 2u log2(e) = x (E0 + E1 x^2)
constexpr float kGeluE1 = kGeluE0 * kGeluK1;
DTF_DEV float gelu_r(float x, float x2) {
  const float y = x * __builtin_fmaf(x2, kGeluE1, kGeluE0);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(y));
}
DTF_DEV float gelu_f(float x) {
  const float r = gelu_r(x, x * x);
  return __builtin_fmaf(-x, r, x);
}
DTF_DEV float gelu_grad(float x) {
  const float x2 = x * x;
  const float r = gelu_r(x, x2);
  const float q = __builtin_fmaf(x2, 6.f * kGeluK0 * kGeluK1, 2.f * kGeluK0);
  return (1.f - r) * __builtin_fmaf(x * r, q, 1.f);
}


#define HIP_CHECK(x)                                                               \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") +    \
                                                   hipGetErrorString(e_) + " @ " + \
                                                   __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)
