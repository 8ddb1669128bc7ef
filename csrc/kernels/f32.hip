// fp32 path of the reference workload (MNIST CNN / MLP at the reference's own precision).
//
// The reference trains in fp32 end to end (dataset.py:93-95 casts to float32; tf.layers default
// dtype), so comparing against its published times needs an fp32 run.  gfx950 has f32-input MFMA
// (v_mfma_f32_16x16x4_f32, exact f32 fma-chain numerics at the f32 vector rate -- guide §3
// "FP32-input MFMA"), so the fp32 path is still matrix-core work:
//
//   * gemm_f32:  C (+)= act(alpha * sum_k A(m, k) B(n, k) + bias[n]) with ARBITRARY element
//     strides for A, B and C: one kernel serves dense fwd (x W^T), data gradient (dz W), weight
//     gradient (dz^T x, accumulated straight into the optimizer's fp32 flat gradient buffer), the
//     MLP template's [in, out] weights and the convolutions below.  64 x 64 block tile, 4 waves of
//     2 x 2 16x16 fragments, BK 16 staged k-major in LDS (conflict-free fragment reads), global
//     loads ordered along whichever operand dimension is contiguous.
//   * convolution = im2col (one pass, zero padding) + gemm_f32; data gradient = gemm_f32 into
//     column space + col2im as a deterministic GATHER (each input pixel sums its taps; no
//     atomics); weight gradient = gemm_f32 over the saved columns.  (MNIST's convs are 0.16 /
//     2.6 GFLOP at batch 128: the column buffer costs less than a second conv kernel family.)
//   * max-pool 2x2 fwd (argmax byte) / bwd, fused ReluGrad + BiasAddGrad, and the templates'
//     clipped-log softmax cross-entropy (templates/00_mnist_replica.py:160-164) fwd + bwd.
#include <stdexcept>

#include "common.h"

typedef __attribute__((ext_vector_type(4))) float f32x4v;

namespace {

struct F32Gemm {
  const float* A; const float* B; float* C; const float* bias;
  int M, N, K;
  long sam, sak, sbn, sbk, scm, scn;
  float alpha;
  int relu, accumulate;
  int kchunk;          // split-K: blockIdx.y covers k in [y * kchunk, (y + 1) * kchunk)
  long slab;           // split-K: partial y goes to C + y * slab (a workspace), plain store
};

constexpr int kFB = 64, kFK = 16, kFPad = 4;

__global__ void __launch_bounds__(256)
gemm_f32_kernel(const F32Gemm g) {
  __shared__ float sA[kFK][kFB + kFPad];
  __shared__ float sB[kFK][kFB + kFPad];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (g.N + kFB - 1) / kFB;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * kFB, n0 = tn * kFB;
  // which way the 4 loads per thread walk: along k when k is the contiguous dimension
  const bool a_kfast = g.sak == 1, b_kfast = g.sbk == 1;

  f32x4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4v){0.f, 0.f, 0.f, 0.f};

  const int kbeg = blockIdx.y * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
  for (int k0 = kbeg; k0 < kend; k0 += kFK) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + e * 256;
      int kk, mm;
      if (a_kfast) { kk = idx % kFK; mm = idx / kFK; } else { mm = idx % kFB; kk = idx / kFB; }
      const int m = m0 + mm, k = k0 + kk;
      sA[kk][mm] = (m < g.M && k < kend) ? g.A[(long)m * g.sam + (long)k * g.sak] : 0.f;
      int kb, nn;
      if (b_kfast) { kb = idx % kFK; nn = idx / kFK; } else { nn = idx % kFB; kb = idx / kFB; }
      const int n = n0 + nn, kx = k0 + kb;
      sB[kb][nn] = (n < g.N && kx < kend) ? g.B[(long)n * g.sbn + (long)kx * g.sbk] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kg = 0; kg < kFK / 4; ++kg) {
      const int kr = kg * 4 + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sA[kr][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = sB[kr][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + (lane & 15);
      if (col >= g.N) continue;
      const float bv = g.bias ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= g.M) continue;
        float v = g.alpha * acc[i][j][r] + bv;
        if (g.relu) v = fmaxf(v, 0.f);
        float* c = g.C + blockIdx.y * g.slab + (long)row * g.scm + (long)col * g.scn;
        *c = g.accumulate ? *c + v : v;
      }
    }
}

// cols[m, t * C + c] = x[n, p * sh + dh_t, q * sw + dw_t, c] (0 outside), m = (n, p, q)
__global__ void __launch_bounds__(256)
im2col_f32_kernel(const float* __restrict__ x, float* __restrict__ cols, int N, int H, int W,
                  int C, int P, int Q, int sh, int sw, int R, int S, int pt, int pl, long total) {
  const long TC = (long)R * S * C;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const long m = idx / TC;
    const int rem = (int)(idx - m * TC);
    const int t = rem / C, c = rem - t * C;
    const int r = t / S, s = t - r * S;
    const int q = (int)(m % Q);
    const long nt = m / Q;
    const int p = (int)(nt % P), n = (int)(nt / P);
    const int h = p * sh + r - pt, w = q * sw + s - pl;
    cols[idx] = ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
                    ? x[(((long)n * H + h) * W + w) * C + c] : 0.f;
  }
}

// dx[n, h, w, c] = sum over taps (r, s) whose output (p, q) exists of dcols[(n, p, q), t*C + c]
__global__ void __launch_bounds__(256)
col2im_f32_kernel(const float* __restrict__ dcols, float* __restrict__ dx, int N, int H, int W,
                  int C, int P, int Q, int sh, int sw, int R, int S, int pt, int pl, long total) {
  const long TC = (long)R * S * C;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int c = (int)(idx % C);
    const long pix = idx / C;
    const int w = (int)(pix % W);
    const long nh = pix / W;
    const int h = (int)(nh % H), n = (int)(nh / H);
    float acc = 0.f;
    for (int r = 0; r < R; ++r) {
      const int ph = h + pt - r;
      if (ph < 0 || ph % sh) continue;
      const int p = ph / sh;
      if (p >= P) continue;
      for (int s = 0; s < S; ++s) {
        const int qw = w + pl - s;
        if (qw < 0 || qw % sw) continue;
        const int q = qw / sw;
        if (q >= Q) continue;
        acc += dcols[(((long)n * P + p) * Q + q) * TC + (long)(r * S + s) * C + c];
      }
    }
    dx[idx] = acc;
  }
}

// 2x2 (kernel k, stride s, VALID) max-pool over NHWC fp32; arg = index of the max in the window
__global__ void __launch_bounds__(256)
maxpool_f32_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, uint8_t* __restrict__ arg,
                       int N, int H, int W, int C, int P, int Q, int k, int s, long total) {
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int c = (int)(idx % C);
    const long pix = idx / C;
    const int q = (int)(pix % Q);
    const long np = pix / Q;
    const int p = (int)(np % P), n = (int)(np / P);
    float best = -__builtin_huge_valf();
    int bi = 0;
    for (int i = 0; i < k; ++i)
      for (int j = 0; j < k; ++j) {
        const int h = p * s + i, w = q * s + j;
        if (h >= H || w >= W) continue;
        const float v = x[(((long)n * H + h) * W + w) * C + c];
        if (v > best || (i == 0 && j == 0)) { best = v; bi = i * k + j; }
      }
    y[idx] = best;
    arg[idx] = (uint8_t)bi;
  }
}

// gather form: each input element finds the (single, s >= k) window it belongs to
__global__ void __launch_bounds__(256)
maxpool_f32_bwd_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ arg,
                       float* __restrict__ dx, int N, int H, int W, int C, int P, int Q, int k,
                       int s, long total) {
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int c = (int)(idx % C);
    const long pix = idx / C;
    const int w = (int)(pix % W);
    const long nh = pix / W;
    const int h = (int)(nh % H), n = (int)(nh / H);
    float g = 0.f;
    const int p = h / s, q = w / s, i = h - p * s, j = w - q * s;
    if (p < P && q < Q && i < k && j < k) {
      const long o = (((long)n * P + p) * Q + q) * C + c;
      if (arg[o] == i * k + j) g = dy[o];
    }
    dx[idx] = g;
  }
}

// dz = relu ? dy * (y > 0) : dy ; ws[slice][col] = partial column sums of dz
__global__ void __launch_bounds__(256)
bias_relu_bwd_f32_kernel(const float* dy, const float* __restrict__ y, float* dz, int T, int N,
                         float* __restrict__ ws, int R, int relu) {
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  __shared__ float red[4][64];
  const int r0 = blockIdx.y * R, r1 = min(T, r0 + R);
  float acc = 0.f;
  if (col < N)
    for (int r = r0 + rg; r < r1; r += 4) {
      float d = dy[(long)r * N + col];
      if (relu && !(y[(long)r * N + col] > 0.f)) d = 0.f;
      dz[(long)r * N + col] = d;
      acc += d;
    }
  red[rg][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rg == 0 && col < N)
    ws[(long)blockIdx.y * N + col] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                     red[2][threadIdx.x] + red[3][threadIdx.x];
}

__global__ void __launch_bounds__(256)
slices_sum_kernel(const float* __restrict__ ws, int S, int N, float* __restrict__ out,
                  int accumulate) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= N) return;
  float t = 0.f;
  for (int k = 0; k < S; ++k) t += ws[(long)k * N + col];
  out[col] = accumulate ? out[col] + t : t;
}

// templates/00_mnist_replica.py:160-164: y = softmax(z); loss = -sum(t * log(clip(y, 1e-10, 1)))
// (a batch SUM); grad wrt z: dL/dy_j = -t_j / y_j where the clip passes (1e-10 <= y_j <= 1),
// dz_i = y_i (g_i - sum_j g_j y_j).  One wave per row.
__global__ void __launch_bounds__(64)
clipped_xent_kernel(const float* __restrict__ z, const float* __restrict__ t, int B, int V,
                    float* __restrict__ row_loss, float* __restrict__ dz, float scale) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* zr = z + (long)b * V;
  const float* tr = t + (long)b * V;
  float mx = -__builtin_huge_valf();
  for (int j = lane; j < V; j += 64) mx = fmaxf(mx, zr[j]);
  mx = wave_max(mx);
  float se = 0.f;
  for (int j = lane; j < V; j += 64) se += __expf(zr[j] - mx);
  se = wave_sum(se);
  float loss = 0.f, gy = 0.f;
  for (int j = lane; j < V; j += 64) {
    const float y = __expf(zr[j] - mx) / se;
    const float yc = fminf(fmaxf(y, 1e-10f), 1.f);
    loss -= tr[j] * __logf(yc);
    const float g = (y >= 1e-10f && y <= 1.f) ? -tr[j] / yc : 0.f;
    gy += g * y;
  }
  loss = wave_sum(loss);
  gy = wave_sum(gy);
  for (int j = lane; j < V; j += 64) {
    const float y = __expf(zr[j] - mx) / se;
    const float yc = fminf(fmaxf(y, 1e-10f), 1.f);
    const float g = (y >= 1e-10f && y <= 1.f) ? -tr[j] / yc : 0.f;
    dz[(long)b * V + j] = scale * y * (g - gy);
  }
  if (lane == 0) row_loss[b] = loss;
}

// C[i] (+)= act(sum_s ws[s * n + i] + bias[col(i)]) in split order (deterministic);
// col(i) = i % N for a row-major C, i / M for a column-major one
__global__ void __launch_bounds__(256)
f32_slab_sum_kernel(const float* __restrict__ ws, float* __restrict__ C, long n, int S,
                    int accumulate, const float* __restrict__ bias, int relu, int M, int N,
                    int colmajor) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float t = 0.f;
    for (int k = 0; k < S; ++k) t += ws[(long)k * n + i];
    if (bias) t += bias[colmajor ? i / M : i % N];
    if (relu) t = fmaxf(t, 0.f);
    C[i] = accumulate ? C[i] + t : t;
  }
}

int grid_for(long total) {
  long g = (total + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

}  // namespace

// Split-K plan: a weight gradient sums over every pixel / token (K = 25088-100352 for MNIST's
// convs) into a handful of output tiles; splitting K keeps >= ~512 blocks in flight.
int dtf_gemm_f32_splits(int M, int N, int K) {
  const long tiles = (long)((M + kFB - 1) / kFB) * ((N + kFB - 1) / kFB);
  if (tiles >= 256 || K < 2048) return 1;
  long s = (512 + tiles - 1) / tiles;
  const long maxs = K / 512;
  if (s > maxs) s = maxs;
  return (int)(s < 1 ? 1 : s);
}

void dtf_gemm_f32(const float* A, const float* B, float* C, const float* bias, int M, int N,
                  int K, long sam, long sak, long sbn, long sbk, long scm, long scn, float alpha,
                  int relu, int accumulate, float* ws, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  const long tiles = (long)((M + kFB - 1) / kFB) * ((N + kFB - 1) / kFB);
  const int S = dtf_gemm_f32_splits(M, N, K);
  if (S == 1) {
    F32Gemm g{A, B, C, bias, M, N, K, sam, sak, sbn, sbk, scm, scn, alpha, relu, accumulate,
              K, 0};
    hipLaunchKernelGGL(gemm_f32_kernel, dim3((unsigned)tiles), dim3(256), 0, st, g);
    return;
  }
  if (!ws) throw std::runtime_error("gemm_f32 split-K needs a workspace");
  // C must be a dense M x N block in either orientation (the slabs reuse its strides)
  if (!((scm == N && scn == 1) || (scm == 1 && scn == M)))
    throw std::runtime_error("gemm_f32 split-K: C must be contiguous");
  int kchunk = (K + S - 1) / S;
  kchunk = (kchunk + kFK - 1) / kFK * kFK;
  const int Sr = (K + kchunk - 1) / kchunk;
  F32Gemm g{A, B, ws, nullptr, M, N, K, sam, sak, sbn, sbk, scm, scn, alpha, 0, 0, kchunk,
            (long)M * N};
  hipLaunchKernelGGL(gemm_f32_kernel, dim3((unsigned)tiles, (unsigned)Sr), dim3(256), 0, st, g);
  // splits that got no K (rounding) were never launched: Sr <= S slabs are summed
  hipLaunchKernelGGL(f32_slab_sum_kernel, dim3(grid_for((long)M * N)), dim3(256), 0, st, ws, C,
                     (long)M * N, Sr, accumulate, bias, relu, M, N, (int)(scm == 1 && N > 1));
}

void dtf_im2col_f32(const float* x, float* cols, int N, int H, int W, int C, int P, int Q, int sh,
                    int sw, int R, int S, int pt, int pl, hipStream_t st) {
  const long total = (long)N * P * Q * R * S * C;
  hipLaunchKernelGGL(im2col_f32_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, cols, N, H, W,
                     C, P, Q, sh, sw, R, S, pt, pl, total);
}

void dtf_col2im_f32(const float* dcols, float* dx, int N, int H, int W, int C, int P, int Q,
                    int sh, int sw, int R, int S, int pt, int pl, hipStream_t st) {
  const long total = (long)N * H * W * C;
  hipLaunchKernelGGL(col2im_f32_kernel, dim3(grid_for(total)), dim3(256), 0, st, dcols, dx, N, H,
                     W, C, P, Q, sh, sw, R, S, pt, pl, total);
}

void dtf_maxpool_f32_fwd(const float* x, float* y, uint8_t* arg, int N, int H, int W, int C,
                         int P, int Q, int k, int s, hipStream_t st) {
  if (s < k) throw std::runtime_error("maxpool_f32: overlapping windows unsupported (s < k)");
  const long total = (long)N * P * Q * C;
  hipLaunchKernelGGL(maxpool_f32_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, y, arg,
                     N, H, W, C, P, Q, k, s, total);
}

void dtf_maxpool_f32_bwd(const float* dy, const uint8_t* arg, float* dx, int N, int H, int W,
                         int C, int P, int Q, int k, int s, hipStream_t st) {
  const long total = (long)N * H * W * C;
  hipLaunchKernelGGL(maxpool_f32_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, dy, arg,
                     dx, N, H, W, C, P, Q, k, s, total);
}

int dtf_bias_relu_bwd_f32_ws_floats(int N) { return 256 * N; }

void dtf_bias_relu_bwd_f32(const float* dy, const float* y, float* dz, int T, int N, float* ws,
                           float* db, int accumulate, int relu, hipStream_t st) {
  if (T <= 0 || N <= 0) return;
  int S = T / 32;
  S = S < 1 ? 1 : (S > 256 ? 256 : S);
  const int R = (T + S - 1) / S;
  hipLaunchKernelGGL(bias_relu_bwd_f32_kernel, dim3((N + 63) / 64, S), dim3(256), 0, st, dy, y,
                     dz, T, N, ws, R, relu);
  if (db)
    hipLaunchKernelGGL(slices_sum_kernel, dim3((N + 255) / 256), dim3(256), 0, st, ws, S, N, db,
                       accumulate);
}

void dtf_clipped_xent(const float* z, const float* t, int B, int V, float* row_loss, float* dz,
                      float scale, hipStream_t st) {
  if (B <= 0) return;
  hipLaunchKernelGGL(clipped_xent_kernel, dim3(B), dim3(64), 0, st, z, t, B, V, row_loss, dz,
                     scale);
}
