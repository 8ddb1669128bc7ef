"""Fused c3 backward kernels (csrc/kernels/conv1x1_bwd.hip) at the ResNet-50 b1984 shapes: time
per call of the stored-dO form and of the lazy form (dO formed from the residual BN's dy, x,
ReLU mask; stage 0 also recomputes x), with the HBM bytes each moves and the rate.

    python tools/c1_bench.py [--batch 1984] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflow_amd.ops import native  # noqa: E402

_K = native.kernels()


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1984)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda"
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for C, hw in ((64, 56), (128, 28)):
        K = 4 * C
        M = a.batch * hw * hw
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(M, C, device=dev, generator=g).bfloat16()
        y = torch.relu(x).contiguous()
        w = (torch.randn(K, C, device=dev, generator=g) / C ** 0.5).bfloat16()
        wt = w.t().contiguous()
        dout = torch.randn(M, K, device=dev, generator=g).bfloat16()
        x3 = torch.randn(M, K, device=dev, generator=g).bfloat16()
        mask = torch.randint(0, 256, (M * K // 8,), device=dev, dtype=torch.uint8)
        stats = torch.rand(4, C, device=dev) + 0.5
        coef = torch.rand(3, K, device=dev)
        dy = torch.empty_like(y)
        for lazy, w16 in ((False, 0), (False, 1), (True, 0), (True, 1)):
            if C != 64 and w16:
                continue
            _K.conv1x1_bwd_set_w16(w16)
            G = (_K.conv1x1_bwd_lazy_blocks(M, C) if lazy else _K.conv1x1_bwd_blocks(M, C))
            wpart = torch.empty(G * K * C, device=dev)
            part = torch.empty(_K.bn_workspace_floats_g(G, C), device=dev)
            common = (wt.data_ptr(), y.data_ptr(), x.data_ptr(), stats[0].data_ptr(),
                      stats[1].data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(),
                      dy.data_ptr(), wpart.data_ptr(), part.data_ptr(), M, C, K)
            if lazy:
                fn = lambda: _K.conv1x1_bwd_lazy(  # noqa: E731
                    dout.data_ptr(), x3.data_ptr(), mask.data_ptr(), coef[0].data_ptr(),
                    coef[1].data_ptr(), coef[2].data_ptr(), *common, w.data_ptr(), st())
                reads_x3 = C != 64                     # stage 0 recomputes x3
                nbytes = M * (K * 2 + (K * 2 if reads_x3 else 0) + K // 8 + C * 6)
            else:
                fn = lambda: _K.conv1x1_bwd(dout.data_ptr(), *common, st())  # noqa: E731
                nbytes = M * (K * 2 + C * 6)
            us = timeit(fn, a.iters)
            print(json.dumps({"probe": "c1_bench", "C": C, "K": K, "M": M, "lazy": lazy, "w16": w16,
                              "blocks": G, "us": round(us, 1), "GB": round(nbytes / 1e9, 2),
                              "TBps": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
