"""3x3 halo data gradients with and without the fused BN-backward sums (conv3x3_halo_kernel BNB)
at the ResNet-50 stage-0/1 shapes: conv -> BN + ReLU -> 3x3 conv, forward + backward, timed per
iteration with the halo-epilogue sums on and off (the reduce pass then runs instead).  Also the
driver for the PMC pass of tools/pmc_halo.sh.

    python tools/halo_bnb_bench.py [--batch 256] [--iters 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflow_amd.ops import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    for H, C in ((56, 64), (28, 128)):
        torch.manual_seed(0)
        x = torch.randn(a.batch, H, H, C, device="cuda").bfloat16()
        w1 = (torch.randn(C, 3, 3, C, device="cuda") / (9 * C) ** 0.5).requires_grad_(True)
        w2 = (torch.randn(C, 3, 3, C, device="cuda") / (9 * C) ** 0.5).requires_grad_(True)
        gamma = (torch.rand(C, device="cuda") + 0.5).requires_grad_(True)
        beta = (torch.randn(C, device="cuda") * 0.1).requires_grad_(True)
        g = None
        for fuse in (True, False, True, False):
            native._FUSE_BN_BWD_HALO = fuse

            def step():
                xi = x.clone().requires_grad_(True)
                y1 = native.conv2d(xi, w1, 1, 1, bn_stats=True)
                z = native.batch_norm(y1, gamma, beta, None, None, True, 0.9, 1e-5, relu=True)
                y2 = native.conv2d(z, w2, 1, 1)
                y2.backward(g if g is not None else torch.ones_like(y2))
            step()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                step()
            e.record()
            torch.cuda.synchronize()
            print(json.dumps({"probe": "halo_bnb", "H": H, "C": C, "batch": a.batch,
                              "fused_bn_sums": fuse,
                              "ms_per_fwd_bwd": round(s.elapsed_time(e) / a.iters, 3)}), flush=True)
        native._FUSE_BN_BWD_HALO = True


if __name__ == "__main__":
    main()
