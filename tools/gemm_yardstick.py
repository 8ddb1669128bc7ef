"""Yardstick: our 1x1-conv forward kernel vs hipBLASLt (torch.mm) on the same NHWC GEMMs.

A stride-1 1x1 conv in NHWC is the plain GEMM Y[M, K] = X[M, C] @ W[K, C]^T; this times both
(HIP events, median) at the ResNet-50 batch-512 shapes so the conv kernel's headroom is known.
"""
import json

import torch

from distributedtensorflow_amd.ops import native


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


SHAPES = [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
          (14, 1024, 256), (7, 512, 2048), (7, 2048, 512), (28, 256, 256), (14, 1024, 1024)]


def main(B=512):
    for H, C, K in SHAPES:
        M = B * H * H
        x = torch.randn(B, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(K, 1, 1, C, device="cuda") * 0.05).bfloat16()
        x2, w2 = x.view(M, C), w.view(K, C)
        t_ours = timeit(lambda: native.conv2d_forward(x, w, 1, 0))
        t_blas = timeit(lambda: torch.mm(x2, w2.t()))
        fl = 2.0 * M * C * K
        print(json.dumps({"H": H, "C": C, "K": K, "M": M, "ours_us": round(t_ours, 1),
                          "blas_us": round(t_blas, 1), "ours_TF": round(fl / t_ours / 1e6, 1),
                          "blas_TF": round(fl / t_blas / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
