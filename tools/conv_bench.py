"""Per-shape roofline table for the ResNet-50 (batch 256) convolutions: our fwd / dgrad / wgrad
kernels timed with HIP events, reported as TFLOP/s, GB/s (compulsory bytes) and the fraction
of the binding roof (2.5 PF/s bf16 dense, ~5 TB/s achievable HBM).

    python tools/conv_bench.py [--batch 256] [--iters 20]
"""
import argparse
import collections
import json

import torch

from distributedtensorflow_amd.ops import native

PEAK_TF = 2500.0
PEAK_BW = 5.0e12   # achievable HBM3E (~8 TB/s theoretical)


def resnet50_convs(B):
    """(name, H, W, C, K, R, stride, pad, count) of every conv (v1.5: stride on the 3x3)."""
    # the stem runs as a 4x4/1 VALID conv on the 115x115x16 space-to-depth image
    # (ops.reference.space_to_depth_operands); the original 7x7/2 form is kept for comparison
    out = [("stem", 224, 224, 3, 64, 7, 2, 3, 0), ("stem_s2d", 115, 115, 16, 64, 4, 1, 0, 1)]
    cin, res = 64, 56
    for si, (n, w) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
        for bi in range(n):
            s = 2 if (bi == 0 and si > 0) else 1
            out.append((f"s{si}b{bi}c1", res, res, cin, w, 1, 1, 0, 1))
            out.append((f"s{si}b{bi}c2", res, res, w, w, 3, s, 1, 1))
            res2 = res // s
            out.append((f"s{si}b{bi}c3", res2, res2, w, 4 * w, 1, 1, 0, 1))
            if bi == 0:
                out.append((f"s{si}b{bi}proj", res, res, cin, 4 * w, 1, s, 0, 1))
            cin, res = 4 * w, res2
    # merge identical shapes
    agg = collections.OrderedDict()
    for name, H, W, C, K, R, s, p, c in out:
        key = (H, W, C, K, R, s, p)
        if key in agg:
            agg[key][1] += c
        else:
            agg[key] = [name, c]
    return [(v[0], *k, v[1]) for k, v in agg.items()]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None, help="comma list of layer names to run")
    ap.add_argument("--kinds", default="fwd,dgrad,wgrad", help="fwd,fwdbn,dgrad,wgrad")
    ap.add_argument("--dma", type=int, default=-1,
                    help="conv kernel choice: -1 auto, 0 register-staged only, 1 LDS-DMA when legal")
    ap.add_argument("--small-k", type=int, default=None,
                    help="conv_set_small_k bitmask (1: one LDS stage for single-K-step convs, "
                         "2: BK 32 for 1x1 convs with C <= 128)")
    ap.add_argument("--wgrad-mode", type=int, default=-1,
                    help="wgrad_set_dma_mode: -1/1 LDS-DMA (narrow 1x4 for Kout <= 64), "
                         "2 LDS-DMA 2x2 only, 0 register-staged")
    ap.add_argument("--wgrad-pp", type=int, default=1,
                    help="wgrad_set_pp: 0 off, n > 0: 256 x 256 ping-pong kernel for Kout, T*C >= 256 "
                         "with a split-K target of n rounds of 256 blocks")
    ap.add_argument("--gemm-pp", type=int, default=0,
                    help="gemm_set_pp bitmask: 1 persistent register-epilogue GEMM for the "
                         "GEMM-routed 1x1 convs, 2 also for the implicit-GEMM convs")
    ap.add_argument("--conv-gemm", type=int, default=1,
                    help="conv_set_gemm bitmask: 1 implicit-GEMM route for Kout >= 256, 2 also "
                         "for 64 < Kout <= 128 (256 x 128 tile)")
    args = ap.parse_args()
    native._K.wgrad_set_pp(args.wgrad_pp)
    native._K.gemm_set_pp(args.gemm_pp)
    native._K.conv_set_gemm(args.conv_gemm)
    native._K.conv_set_dma_mode(args.dma)
    native._K.wgrad_set_dma_mode(args.wgrad_mode)
    if args.small_k is not None:
        native._K.conv_set_small_k(args.small_k)
    only = set(args.only.split(",")) if args.only else None
    kinds = set(args.kinds.split(","))
    B = args.batch
    rows, tot = [], collections.Counter()
    for name, H, W, C, K, R, s, p, cnt in resnet50_convs(B):
        if only and name not in only:
            continue
        C = -(-C // 8) * 8          # the op zero-pads C=3 (stem) to 8 channels
        x = torch.randn(B, H, W, C, device="cuda").bfloat16()
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
        y = native.conv2d_forward(x, w, s, p)
        P, Q = y.shape[1], y.shape[2]
        dy = torch.randn_like(y)
        flops = 2.0 * B * P * Q * K * R * R * C
        xb, yb, wb = x.numel() * 2, y.numel() * 2, w.numel() * 2
        # fwdbn: the training-step forward, BatchNorm partial sums fused into the epilogue
        part = torch.empty(((B * P * Q) // 64 + 2) * 2 * K, device="cuda", dtype=torch.float32)
        cases = [("fwd", lambda: native.conv2d_forward(x, w, s, p), xb + yb + wb),
                 ("fwdbn", lambda: native.conv2d_forward(x, w, s, p, stats=part), xb + yb + wb)]
        # the stem's input is the image: training never computes its data gradient, so the
        # stem rows carry no dgrad (it would only inflate the per-step totals)
        if C % 8 == 0 and not name.startswith("stem"):
            cases.append(("dgrad", lambda: native.conv2d_dgrad(dy, w, x.shape, s, p),
                          xb + yb + wb))
        cases.append(("wgrad", lambda: native.conv2d_wgrad(x, dy, w.shape, s, p),
                      xb + yb + 2 * wb))
        for kind, fn, nbytes in cases:
            if kind not in kinds:
                continue
            t = timeit(fn, args.iters)
            tf = flops / t / 1e12
            bw = nbytes / t
            roof = max(flops / (PEAK_TF * 1e12), nbytes / PEAK_BW)
            rows.append({"layer": name, "kind": kind, "shape": f"{H}x{W}x{C}->{K} r{R} s{s}",
                         "count": cnt, "us": round(t * 1e6, 1), "tflops": round(tf, 1),
                         "GBps": round(bw / 1e9), "roof_frac": round(roof / t, 3)})
            tot[kind] += t * cnt
            tot["roof_" + kind] += roof * cnt
    for r in rows:
        print(json.dumps(r), flush=True)
    summ = {k: round(v * 1e3, 3) for k, v in tot.items()}
    print(json.dumps({"total_ms": summ}), flush=True)


if __name__ == "__main__":
    main()
