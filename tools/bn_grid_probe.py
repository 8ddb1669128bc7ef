"""Grid size of the BatchNorm row sweeps on the ResNet-50 b1984 shapes.

The apply / backward-apply sweeps are grid-stride loops whose grid the launcher sizes from the
row count (up to 8 blocks per CU); the reduce passes target a block count.  This sweeps both
knobs (``bn_set_grid_cap``, ``bn_set_stats_blocks``) per kernel and shape and prints one JSON line
per (kernel, shape, knob) with the time per launch.

    python tools/bn_grid_probe.py [--batch 1984] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflow_amd.ops import native  # noqa: E402

_K = native.kernels()

SHAPES = [(56 * 56, 64), (56 * 56, 256), (28 * 28, 128), (28 * 28, 512), (14 * 14, 256),
          (14 * 14, 1024), (7 * 7, 512), (7 * 7, 2048)]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1984)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for pix, C in SHAPES:
        M = args.batch * pix
        x = torch.randn(M, C, device=dev).to(bf)
        dy = torch.randn(M, C, device=dev).to(bf)
        res = torch.randn(M, C, device=dev).to(bf)
        out = torch.empty_like(x)
        out2 = torch.empty_like(x)
        mask = torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
        co = torch.randn(5, C, device=dev) * 0.1
        sc, sh = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        mean, inv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        gb = M * C * 2 / 1e9
        sweeps = {
            # name: (fn, GB moved)
            "apply_relu": (lambda: _K.bn_apply(x.data_ptr(), 0, out.data_ptr(), sc.data_ptr(),
                                               sh.data_ptr(), M, C, 1, st(), 0), 2 * gb),
            "apply_res_mask": (lambda: _K.bn_apply(x.data_ptr(), res.data_ptr(), out.data_ptr(),
                                                   sc.data_ptr(), sh.data_ptr(), M, C, 1, st(),
                                                   mask.data_ptr()), 3 * gb + gb / 16),
            "bwd_apply_relu_x": (lambda: _K.bn_bwd_apply(
                dy.data_ptr(), 0, x.data_ptr(), co[2].data_ptr(), co[3].data_ptr(),
                co[4].data_ptr(), out.data_ptr(), 0, M, C, 1, st(), sc.data_ptr(), sh.data_ptr(),
                0), 3 * gb),
            "bwd_apply_mask_dres": (lambda: _K.bn_bwd_apply(
                dy.data_ptr(), 0, x.data_ptr(), co[2].data_ptr(), co[3].data_ptr(),
                co[4].data_ptr(), out.data_ptr(), out2.data_ptr(), M, C, 1, st(), 0, 0,
                mask.data_ptr()), 4 * gb + gb / 16),
        }
        for name, (fn, gbytes) in sweeps.items():
            for cap in (0, 1536, 1024, 768, 512, 384, 256):
                _K.bn_set_grid_cap(cap)
                ms = timed(fn, args.reps)
                print(json.dumps({"probe": "bn_grid", "kernel": name, "M": M, "C": C,
                                  "grid_cap": cap, "ms": round(ms, 4),
                                  "TBps": round(gbytes / ms, 2)}), flush=True)
        _K.bn_set_grid_cap(0)
        for blocks in (1024, 768, 512, 384, 256):
            _K.bn_set_stats_blocks(blocks)
            part = torch.empty(_K.bn_workspace_floats(M, C), device=dev, dtype=torch.float32)
            fn = (lambda: _K.bn_bwd_reduce(dy.data_ptr(), 0, x.data_ptr(), mean.data_ptr(),
                                           inv.data_ptr(), M, C, 1, part.data_ptr(), st(),
                                           sc.data_ptr(), sh.data_ptr(), 0))
            ms = timed(fn, args.reps)
            print(json.dumps({"probe": "bn_grid", "kernel": "bwd_reduce_relu_x", "M": M, "C": C,
                              "stats_blocks": blocks, "ms": round(ms, 4),
                              "TBps": round(2 * gb / ms, 2)}), flush=True)
        _K.bn_set_stats_blocks(1024)
        del x, dy, res, out, out2, mask
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
