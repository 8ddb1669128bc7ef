"""Can a memory-bound BatchNorm pass and a compute-bound conv weight gradient share the chip?

Times, on real ResNet-50 b1984 shapes:
  A  = the weight gradient of a 3x3 conv (compute-bound MFMA kernel), alone;
  B  = a BatchNorm backward apply sweep (HBM-bound), alone, at several grid caps;
  AB = both, A on one stream and B on another, launched interleaved.
overlap = (A + B - AB) / min(A, B): 0 = the two kernels serialize, 1 = the shorter one is fully
hidden.  Prints one JSON line per configuration.

    python tools/overlap_probe.py [--batch 1984] [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflow_amd.ops import native  # noqa: E402

_K = native.kernels()


def timed(fn, reps):
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
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda")
    B = args.batch
    bf = torch.bfloat16
    # compute-bound: s2b1c2 weight gradient (14x14x256 -> 256, 3x3) and s1b1c2 (28x28x128)
    wg = {}
    for name, hw, c in (("s2_3x3", 14, 256), ("s1_3x3", 28, 128)):
        x = torch.randn(B, hw, hw, c, device=dev).to(bf)
        dy = torch.randn(B, hw, hw, c, device=dev).to(bf)
        out = torch.zeros(c, 3, 3, c, device=dev)
        wg[name] = (lambda x=x, dy=dy, out=out, c=c:
                    native.conv2d_wgrad(x, dy, (c, 3, 3, c), 1, 1, out=out))
    # memory-bound: BN backward apply over a stage-2 block output [B*28*28, 512] (relu from x)
    M, C = B * 28 * 28, 512
    x = torch.randn(M, C, device=dev).to(bf)
    dy = torch.randn(M, C, device=dev).to(bf)
    dx = torch.empty_like(x)
    co = torch.randn(5, C, device=dev) * 0.1
    sc, sh = torch.ones(C, device=dev), torch.zeros(C, device=dev)

    def bn():
        _K.bn_bwd_apply(dy.data_ptr(), 0, x.data_ptr(), co[2].data_ptr(), co[3].data_ptr(),
                        co[4].data_ptr(), dx.data_ptr(), 0, M, C, 1,
                        torch.cuda.current_stream().cuda_stream, sc.data_ptr(), sh.data_ptr(), 0)

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for name, fa in wg.items():
        for fn in (fa, bn):
            timed(fn, 2)
        ta = timed(fa, args.reps)
        for cap in (0, 1024, 512, 256, 128, 64):
            _K.bn_set_grid_cap(cap)
            timed(bn, 2)
            tb = timed(bn, args.reps)

            def both():
                cur = torch.cuda.current_stream()
                s1.wait_stream(cur)
                s2.wait_stream(cur)
                for _ in range(args.reps):
                    with torch.cuda.stream(s1):
                        fa()
                    with torch.cuda.stream(s2):
                        bn()
                cur.wait_stream(s1)
                cur.wait_stream(s2)
            timed(both, 1)
            tab = timed(both, 1) / args.reps
            print(json.dumps({"probe": "overlap", "wgrad": name, "bn_grid_cap": cap,
                              "wgrad_ms": round(ta, 4), "bn_ms": round(tb, 4),
                              "both_ms": round(tab, 4), "serial_ms": round(ta + tb, 4),
                              "overlap": round((ta + tb - tab) / min(ta, tb), 3)}), flush=True)
        _K.bn_set_grid_cap(0)


if __name__ == "__main__":
    main()
