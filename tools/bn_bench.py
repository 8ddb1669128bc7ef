"""BatchNorm streaming-kernel bandwidth at the ResNet-50 shapes (batch 512 by default).

    python tools/bn_bench.py [--batch 512] [--out profiles/r1_bn_bandwidth_b512.jsonl]

For every distinct (H*W, C, residual) BN of ResNet-50 v1.5 it times bn_apply, bn_bwd_reduce and
bn_bwd_apply (HIP events, median of 20) and reports the bytes each moves and the achieved TB/s,
next to a plain device copy of the same tensor (torch ``copy_``) as the attainable-bandwidth
yardstick.  Per-step totals weight each shape by how often ResNet-50 runs it.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflow_amd.ops import native as nat  # noqa: E402

K = nat.kernels()

# (H*W, C, residual+relu, relu, count per step) -- ResNet-50 v1.5 at 224x224
SHAPES = [
    (112 * 112, 64, False, True, 1),      # stem
    (56 * 56, 64, False, True, 6),        # stage 1 bn1/bn2 (3 blocks x 2)
    (56 * 56, 256, True, True, 3),        # stage 1 bn3 (+res)
    (56 * 56, 256, False, False, 1),      # stage 1 projection
    (56 * 56, 128, False, True, 1),       # stage 2 block 1 bn1
    (28 * 28, 128, False, True, 7),
    (28 * 28, 512, True, True, 4),
    (28 * 28, 512, False, False, 1),
    (28 * 28, 256, False, True, 1),
    (14 * 14, 256, False, True, 11),
    (14 * 14, 1024, True, True, 6),
    (14 * 14, 1024, False, False, 1),
    (14 * 14, 512, False, True, 1),
    (7 * 7, 512, False, True, 5),
    (7 * 7, 2048, True, True, 3),
    (7 * 7, 2048, False, False, 1),
]


def timeit(fn, iters=20):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default=None)
    ap.add_argument("--nt", type=int, default=7, help="bn_set_nt bitmask: 1 apply, 2 bwd apply, 4 reduce")
    args = ap.parse_args()
    K.bn_set_nt(args.nt)
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    rows, tot = [], {"apply": 0.0, "reduce": 0.0, "bwd_apply": 0.0, "copy": 0.0}
    for hw, C, res, relu, cnt in SHAPES:
        M = args.batch * hw
        E = M * C
        x = (torch.randn(M, C, device=dev) * 2).to(torch.bfloat16)
        r = torch.randn_like(x) if res else None
        dy = torch.randn_like(x)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        mask = torch.empty(E // 8, device=dev, dtype=torch.uint8) if res else None
        co = torch.rand(8, C, device=dev)
        part = torch.empty(K.bn_workspace_floats(M, C), device=dev)
        sc, sh = co[0].data_ptr(), co[1].data_ptr()
        t_apply = timeit(lambda: K.bn_apply(x.data_ptr(), nat._p(r), y.data_ptr(), sc, sh, M, C,
                                            int(relu), st, nat._p(mask)))
        mx = relu and not res
        t_red = timeit(lambda: K.bn_bwd_reduce(dy.data_ptr(), 0, x.data_ptr(), co[2].data_ptr(),
                                               co[3].data_ptr(), M, C, int(relu), part.data_ptr(),
                                               st, sc if mx else 0, sh if mx else 0,
                                               nat._p(mask)))
        t_bwd = timeit(lambda: K.bn_bwd_apply(dy.data_ptr(), 0, x.data_ptr(), co[4].data_ptr(),
                                              co[5].data_ptr(), co[6].data_ptr(), dx.data_ptr(),
                                              0, M, C, int(relu), st, sc if mx else 0,
                                              sh if mx else 0, nat._p(mask)))
        t_copy = timeit(lambda: y.copy_(x))
        mb = E // 8 if res else 0
        b_apply = 2 * E * (2 + (1 if res else 0)) + mb
        b_red = 2 * E * 2 + mb
        b_bwd = 2 * E * 3 + mb
        rec = {"HW": hw, "C": C, "res": res, "relu": relu, "count": cnt, "M": M,
               "apply_us": round(t_apply, 1), "apply_TBps": round(b_apply / t_apply / 1e6, 2),
               "reduce_us": round(t_red, 1), "reduce_TBps": round(b_red / t_red / 1e6, 2),
               "bwd_apply_us": round(t_bwd, 1), "bwd_apply_TBps": round(b_bwd / t_bwd / 1e6, 2),
               "copy_us": round(t_copy, 1), "copy_TBps": round(4 * E / t_copy / 1e6, 2)}
        rows.append(rec)
        tot["apply"] += cnt * t_apply
        tot["reduce"] += cnt * t_red
        tot["bwd_apply"] += cnt * t_bwd
        tot["copy"] += cnt * t_copy
        print(json.dumps(rec), flush=True)
        del x, r, dy, y, dx, mask, part
    summ = {"summary_ms_per_step": {k: round(v / 1e3, 3) for k, v in tot.items()},
            "batch": args.batch}
    print(json.dumps(summ), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            for rec in rows + [summ]:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
