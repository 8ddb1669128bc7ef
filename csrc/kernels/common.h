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

#define HIP_CHECK(x)                                                               \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") +    \
                                                   hipGetErrorString(e_) + " @ " + \
                                                   __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)
