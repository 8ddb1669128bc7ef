"""Probe: 1x1 stride-1 conv weight gradients as a plain GEMM (dW[K,C] = dY^T X) on hipBLASLt
(torch.mm out_dtype=float32) vs the implicit-GEMM wgrad kernel.  Prints one JSON line per shape."""
import json
import sys

import torch

from distributedtensorflow_amd.ops import native


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    shapes = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512),
              (28, 512, 128), (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (14, 1024, 512),
              (7, 512, 2048), (7, 2048, 512)]
    for H, C, K in shapes:
        M = B * H * H
        x = torch.randn(B, H, H, C, device="cuda").bfloat16()
        dy = torch.randn(B, H, H, K, device="cuda").bfloat16()
        w = torch.zeros(K, 1, 1, C, device="cuda").bfloat16()
        tgt = torch.zeros(K, C, device="cuda")
        ours = timeit(lambda: native.conv2d_wgrad(x, dy, w.shape, 1, 0, out=tgt.view(K, 1, 1, C)))
        d2, x2 = dy.view(M, K), x.view(M, C)
        blas = timeit(lambda: torch.mm(d2.t(), x2, out_dtype=torch.float32))
        blas_acc = timeit(lambda: tgt.add_(torch.mm(d2.t(), x2, out_dtype=torch.float32)))
        ref = (d2.float().t() @ x2.float())
        got = torch.mm(d2.t(), x2, out_dtype=torch.float32)
        tgt.zero_()
        native.conv2d_wgrad(x, dy, w.shape, 1, 0, out=tgt.view(K, 1, 1, C))
        err_b = ((got - ref).norm() / ref.norm()).item()
        err_o = ((tgt - ref).norm() / ref.norm()).item()
        print(json.dumps({"H": H, "C": C, "K": K, "M": M, "ours_us": round(ours, 1),
                          "blas_us": round(blas, 1), "blas_acc_us": round(blas_acc, 1),
                          "err_blas": err_b, "err_ours": err_o}), flush=True)


if __name__ == "__main__":
    main()
