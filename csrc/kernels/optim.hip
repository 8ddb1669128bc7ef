// Fused optimizer updates over FLAT fp32 buffers (all parameters of a strategy live in one
// contiguous master buffer, so one launch updates the whole model — no multi-tensor lists).
//
// TF-exact update math:
//   Momentum (tf.train.MomentumOptimizer):  a = mu*a + g;  p -= lr*a   (nesterov: p -= lr*(g + mu*a))
//   Adam     (tf.train.AdamOptimizer):      lr_t = lr*sqrt(1-b2^t)/(1-b1^t)
//                                           m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2
//                                           p -= lr_t * m / (sqrt(v) + eps)   <- eps OUTSIDE the
//                                           bias correction, unlike torch.optim.Adam
//   Adagrad  (tf.train.AdagradOptimizer):   acc += g^2; p -= lr * g * rsqrt(acc)   (acc0 = 0.1)
//   LAMB     (per-tensor trust ratio):      u = m_hat/(sqrt(v_hat)+eps) + wd*p;
//                                           p -= lr * (|p|/|u|) * u
// Every kernel optionally writes the bf16 compute shadow of p in the same pass (saves the
// separate cast of the fp32 master every step) and flags non-finite gradients.
// Hyper-parameters that change per step (lr, lr_t) are read from DEVICE memory so a captured
// hipGraph replays correctly.
#include "common.h"

namespace {
constexpr int kT = 256;

DTF_DEV void flag_nonfinite(int* flag, float g) {
  if (flag && !isfinite(g)) atomicOr(flag, 1);
}

__global__ void __launch_bounds__(kT)
sgd_momentum_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ a,
                    bf16_t* __restrict__ shadow, long n, const float* __restrict__ lr_ptr,
                    float momentum, float wd, float gscale, int nesterov, int* nonfinite) {
  const float lr = *lr_ptr;
  const long n4 = n >> 2;
  for (long i = (long)blockIdx.x * kT + threadIdx.x; i < n4; i += (long)gridDim.x * kT) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 av = reinterpret_cast<float4*>(a)[i];
    float pp[4] = {pv.x, pv.y, pv.z, pv.w};
    const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    float aa[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      flag_nonfinite(nonfinite, gg[j]);
      const float gr = gg[j] * gscale + wd * pp[j];
      aa[j] = momentum * aa[j] + gr;
      pp[j] -= lr * (nesterov ? gr + momentum * aa[j] : aa[j]);
    }
    reinterpret_cast<float4*>(p)[i] = make_float4(pp[0], pp[1], pp[2], pp[3]);
    reinterpret_cast<float4*>(a)[i] = make_float4(aa[0], aa[1], aa[2], aa[3]);
    if (shadow) {
      uint2 s;
      s.x = pack2(pp[0], pp[1]);
      s.y = pack2(pp[2], pp[3]);
      reinterpret_cast<uint2*>(shadow)[i] = s;
    }
  }
  // scalar tail
  for (long i = n4 * 4 + (long)blockIdx.x * kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) {
    flag_nonfinite(nonfinite, g[i]);
    const float gr = g[i] * gscale + wd * p[i];
    a[i] = momentum * a[i] + gr;
    p[i] -= lr * (nesterov ? gr + momentum * a[i] : a[i]);
    if (shadow) shadow[i] = f2bf(p[i]);
  }
}

__global__ void __launch_bounds__(kT)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
            float* __restrict__ v, bf16_t* __restrict__ shadow, long n,
            const float* __restrict__ lr_t_ptr, float b1, float b2, float eps, float wd,
            float gscale, int* nonfinite) {
  const float lr_t = *lr_t_ptr;
  for (long i = (long)blockIdx.x * kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) {
    const float gr0 = g[i];
    flag_nonfinite(nonfinite, gr0);
    const float gr = gr0 * gscale;
    const float mi = b1 * m[i] + (1.f - b1) * gr;
    const float vi = b2 * v[i] + (1.f - b2) * gr * gr;
    m[i] = mi;
    v[i] = vi;
    float pi = p[i];
    pi -= lr_t * mi / (sqrtf(vi) + eps) + (wd != 0.f ? lr_t * wd * pi : 0.f);
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

__global__ void __launch_bounds__(kT)
adagrad_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ acc,
               bf16_t* __restrict__ shadow, long n, const float* __restrict__ lr_ptr,
               float gscale, int* nonfinite) {
  const float lr = *lr_ptr;
  for (long i = (long)blockIdx.x * kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) {
    const float gr0 = g[i];
    flag_nonfinite(nonfinite, gr0);
    const float gr = gr0 * gscale;
    const float ai = acc[i] + gr * gr;
    acc[i] = ai;
    const float pi = p[i] - lr * gr * rsqrtf(ai);
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

// ---- LAMB: chunk table entries {segment, start, len}; norms[seg] = {sum p^2, sum u^2}
struct Chunk { int seg; int len; long start; };

__global__ void __launch_bounds__(kT)
lamb_phase1_kernel(const float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                   float* __restrict__ v, const Chunk* __restrict__ chunks,
                   const float* __restrict__ hyper, float b1, float b2, float eps,
                   const float* __restrict__ wd_seg, float gscale,
                   float* __restrict__ norms, int* nonfinite) {
  // hyper[0] = 1/(1-b1^t), hyper[1] = 1/(1-b2^t)
  __shared__ float red[2][kT / 64];
  const Chunk c = chunks[blockIdx.x];
  const float bc1 = hyper[0], bc2 = hyper[1];
  const float wd = wd_seg[c.seg];
  float sp = 0.f, su = 0.f;
  for (int j = threadIdx.x; j < c.len; j += kT) {
    const long i = c.start + j;
    const float gr0 = g[i];
    flag_nonfinite(nonfinite, gr0);
    const float gr = gr0 * gscale;
    const float mi = b1 * m[i] + (1.f - b1) * gr;
    const float vi = b2 * v[i] + (1.f - b2) * gr * gr;
    m[i] = mi;
    v[i] = vi;
    const float pi = p[i];
    const float u = (mi * bc1) / (sqrtf(vi * bc2) + eps) + wd * pi;
    g[i] = u;   // the gradient buffer is consumed: reuse it for the update direction
    sp += pi * pi;
    su += u * u;
  }
  sp = wave_sum(sp);
  su = wave_sum(su);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = sp; red[1][w] = su; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < kT / 64; ++k) { a += red[0][k]; b += red[1][k]; }
    atomicAdd(&norms[2 * c.seg], a);
    atomicAdd(&norms[2 * c.seg + 1], b);
  }
}

__global__ void __launch_bounds__(kT)
lamb_phase2_kernel(float* __restrict__ p, const float* __restrict__ u,
                   bf16_t* __restrict__ shadow, const Chunk* __restrict__ chunks,
                   const float* __restrict__ lr_ptr, const float* __restrict__ norms) {
  const Chunk c = chunks[blockIdx.x];
  const float pn = sqrtf(norms[2 * c.seg]), un = sqrtf(norms[2 * c.seg + 1]);
  const float trust = (pn > 0.f && un > 0.f) ? pn / un : 1.f;
  const float step = *lr_ptr * trust;
  for (int j = threadIdx.x; j < c.len; j += kT) {
    const long i = c.start + j;
    const float pi = p[i] - step * u[i];
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

__global__ void __launch_bounds__(kT)
sumsq_kernel(const float* __restrict__ x, long n, float* __restrict__ out) {
  __shared__ float red[kT / 64];
  float s = 0.f;
  for (long i = (long)blockIdx.x * kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) {
    const float v = x[i];
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < kT / 64; ++k) t += red[k];
    atomicAdd(out, t);
  }
}

__global__ void __launch_bounds__(kT)
cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * kT + threadIdx.x; i < n; i += (long)gridDim.x * kT)
    y[i] = f2bf(x[i]);
}

inline int grid_for(long n, int per_thread = 1) {
  long g = (n / per_thread + kT - 1) / kT;
  if (g > 2048) g = 2048;
  return (int)(g < 1 ? 1 : g);
}
}  // namespace

void dtf_sgd_momentum(float* p, const float* g, float* a, bf16_t* shadow, long n,
                      const float* lr_ptr, float momentum, float wd, float gscale, int nesterov,
                      int* nonfinite, hipStream_t st) {
  hipLaunchKernelGGL(sgd_momentum_kernel, dim3(grid_for(n, 4)), dim3(kT), 0, st, p, g, a, shadow, n,
                     lr_ptr, momentum, wd, gscale, nesterov, nonfinite);
}

void dtf_adam(float* p, const float* g, float* m, float* v, bf16_t* shadow, long n,
              const float* lr_t_ptr, float b1, float b2, float eps, float wd, float gscale,
              int* nonfinite, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(kT), 0, st, p, g, m, v, shadow, n,
                     lr_t_ptr, b1, b2, eps, wd, gscale, nonfinite);
}

void dtf_adagrad(float* p, const float* g, float* acc, bf16_t* shadow, long n,
                 const float* lr_ptr, float gscale, int* nonfinite, hipStream_t st) {
  hipLaunchKernelGGL(adagrad_kernel, dim3(grid_for(n)), dim3(kT), 0, st, p, g, acc, shadow, n,
                     lr_ptr, gscale, nonfinite);
}

void dtf_lamb(float* p, float* g, float* m, float* v, bf16_t* shadow, const void* chunks,
              int nchunks, const float* hyper, const float* lr_ptr, float b1, float b2,
              float eps, const float* wd_seg, float gscale, float* norms, int* nonfinite,
              hipStream_t st) {
  hipLaunchKernelGGL(lamb_phase1_kernel, dim3(nchunks), dim3(kT), 0, st, p, g, m, v,
                     (const Chunk*)chunks, hyper, b1, b2, eps, wd_seg, gscale, norms, nonfinite);
  hipLaunchKernelGGL(lamb_phase2_kernel, dim3(nchunks), dim3(kT), 0, st, p, g, shadow,
                     (const Chunk*)chunks, lr_ptr, norms);
}

int dtf_lamb_chunk_bytes() { return (int)sizeof(Chunk); }

void dtf_sumsq(const float* x, long n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid_for(n)), dim3(kT), 0, st, x, n, out);
}

void dtf_cast_f32_bf16(const float* x, bf16_t* y, long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n)), dim3(kT), 0, st, x, y, n);
}
