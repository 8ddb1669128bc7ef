// Fused sparse softmax cross-entropy forward+backward.
// TF semantics (run_mnist_distributed.py:113): loss = mean_b(-log softmax(logits_b)[label_b]);
// the gradient (softmax - onehot) / B is produced in the same pass (one wave per row; the
// row max / sum use 64-lane shuffles) and cached for the backward.
#include "common.h"

namespace {
template <typename LT>
__global__ void __launch_bounds__(256)
xent_kernel(const float* __restrict__ logits, const LT* __restrict__ labels, int B, int V,
            float* __restrict__ loss_rows, float* __restrict__ grad, float grad_scale) {
  const int wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= B) return;
  const float* row = logits + (long)wave * V;
  float mx = -INFINITY;
  for (int i = lane; i < V; i += 64) mx = fmaxf(mx, row[i]);
  mx = wave_max(mx);
  float s = 0.f;
  for (int i = lane; i < V; i += 64) s += __expf(row[i] - mx);
  s = wave_sum(s);
  const float lse = mx + __logf(s);
  const int lab = (int)labels[wave];
  if (lane == 0) loss_rows[wave] = lse - row[lab];
  if (grad) {
    const float inv = 1.f / s;
    float* g = grad + (long)wave * V;
    for (int i = lane; i < V; i += 64) {
      float p = __expf(row[i] - mx) * inv;
      g[i] = (p - (i == lab ? 1.f : 0.f)) * grad_scale;
    }
  }
}
}  // namespace

void dtf_softmax_xent(const float* logits, const void* labels, int label_bytes, int B, int V,
                      float* loss_rows, float* grad, float grad_scale, hipStream_t st) {
  const int blocks = (B * 64 + 255) / 256;
  if (label_bytes == 8)
    hipLaunchKernelGGL(xent_kernel<int64_t>, dim3(blocks), dim3(256), 0, st, logits,
                       (const int64_t*)labels, B, V, loss_rows, grad, grad_scale);
  else
    hipLaunchKernelGGL(xent_kernel<int32_t>, dim3(blocks), dim3(256), 0, st, logits,
                       (const int32_t*)labels, B, V, loss_rows, grad, grad_scale);
}
