"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip) vs hipBLASLt (torch) on the framework's dense
shapes: accuracy against an fp32 reference and HIP-event time per call.

    python tools/gemm_bench.py [--iters 20] [--out gemm.jsonl]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributedtensorflow_amd.ops import native  # noqa: E402

T = 512 * 128
SHAPES = [  # (name, M, N, K): C = A . B^T
    ("bert_qkv_fwd", T, 2304, 768), ("bert_attnout_fwd", T, 768, 768),
    ("bert_ffn1_fwd", T, 3072, 768), ("bert_ffn2_fwd", T, 768, 3072),
    ("bert_qkv_dgrad", T, 768, 2304), ("bert_ffn1_dgrad", T, 768, 3072),
    ("bert_ffn2_dgrad", T, 3072, 768),
    ("bert_mlm_logits", 10240, 30528, 768), ("bert_mlm_dgrad", 10240, 768, 30528),
    ("resnet_fc", 1280, 1000 + 8, 2048), ("mnist_dense", 128, 1024, 3136),
    ("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192),
]


# ResNet-50 1x1 stride-1 convs at batch 1280 as GEMMs: (name, H*W, C, Kout)
RESNET_1X1 = [("s0c1", 3136, 64, 64), ("s0c3", 3136, 64, 256), ("s0b1c1", 3136, 256, 64),
              ("s1b0c1", 3136, 256, 128), ("s1c3", 784, 128, 512), ("s1b1c1", 784, 512, 128),
              ("s2b0c1", 784, 512, 256), ("s2c3", 196, 256, 1024), ("s2b1c1", 196, 1024, 256),
              ("s3b0c1", 196, 1024, 512), ("s3c3", 49, 512, 2048), ("s3b1c1", 49, 2048, 512)]


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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--resnet1x1", type=int, default=0,
                    help="batch: time the ResNet-50 1x1 convs as GEMMs next to the conv kernel")
    ap.add_argument("--dbg", default="0",
                    help="comma list of gemm_set_dbg values to time (kernel experiments)")
    ap.add_argument("--variants", default="0",
                    help="comma list of gemm.hip pipeline variants to time (gemm_set_variant)")
    ap.add_argument("--shapes", default=None,
                    help="extra comma list of MxNxK GEMM shapes (e.g. 388864x1024x256)")
    ap.add_argument("--stagger", default="1:-1",
                    help="comma list of mode:iters start staggers for the OCC-2 variant 12 "
                         "(gemm_set_stagger; -1 iters = auto)")
    a = ap.parse_args()
    rows = []
    if a.resnet1x1:
        for name, hw, C, Kout in RESNET_1X1:
            M = a.resnet1x1 * hw
            g = torch.Generator(device="cuda").manual_seed(0)
            x = torch.randn(M, C, device="cuda", generator=g).bfloat16()
            w = (torch.randn(Kout, C, device="cuda", generator=g) / C ** 0.5).bfloat16()
            x4 = x.view(a.resnet1x1, hw, 1, C)
            w4 = w.view(Kout, 1, 1, C)
            t_conv = timeit(lambda: native.conv2d_forward(x4, w4, 1, 0), a.iters)
            fl = 2.0 * M * Kout * C
            # the training path: conv + fused BN statistics, routed (GEMM) vs conv kernel
            native._CONV_GEMM = True
            t_route = timeit(lambda: native.conv2d(x4, w4, 1, 0, bn_stats=True), a.iters)
            native._CONV_GEMM = False
            t_conv_st = timeit(lambda: native.conv2d(x4, w4, 1, 0, bn_stats=True), a.iters)
            native._CONV_GEMM = True
            rec = {"shape": f"resnet1x1_{name}_bnstats", "routed_us": round(t_route * 1e6, 1),
                   "conv_kernel_us": round(t_conv_st * 1e6, 1),
                   "speedup": round(t_conv_st / t_route, 3)}
            if C in (64, 128, 256) and Kout % 64 == 0:
                # the row-streaming GEMM with the BN statistics epilogue, forced
                ws = torch.empty(native._K.gemm_tile_rows(M) * 2 * Kout, device="cuda")
                native._K.gemm_set_variant(13)
                t_s = timeit(lambda: native.gemm_nt(x, w, stats=ws), a.iters)
                native._K.gemm_set_variant(-1)
                rec["stream_us"] = round(t_s * 1e6, 1)
                rec["stream_speedup"] = round(t_conv_st / t_s, 3)
            print(json.dumps(rec), flush=True)
            for v in [int(x) for x in a.variants.split(",")]:
                if v == 13 and not (C in (64, 128, 256) and Kout % 64 == 0):
                    continue
                native._K.gemm_set_variant(v)
                t_g = timeit(lambda: native.gemm_nt(x, w), a.iters)
                row = {"shape": f"resnet1x1_{name}", "variant": v, "M": M, "N": Kout, "K": C,
                       "gemm_us": round(t_g * 1e6, 1), "conv_us": round(t_conv * 1e6, 1),
                       "gemm_tflops": round(fl / t_g / 1e12, 1),
                       "conv_tflops": round(fl / t_conv / 1e12, 1),
                       "gemm_speedup_vs_conv": round(t_conv / t_g, 3)}
                rows.append(row)
                print(json.dumps(row), flush=True)
            native._K.gemm_set_variant(-1)
            del x, w
            torch.cuda.empty_cache()
        SHAPES_RUN = []
    else:
        SHAPES_RUN = SHAPES
    if a.shapes:
        SHAPES_RUN = [(f"m{sh}", *[int(v) for v in sh.split("x")]) for sh in a.shapes.split(",")]
    for name, M, N, K in SHAPES_RUN:
        if a.only and name not in a.only.split(","):
            continue
        g = torch.Generator(device="cuda").manual_seed(0)
        A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
        ref = torch.nn.functional.linear(A, B)
        sub = slice(0, min(M, 2048))
        exact = A[sub].float() @ B.float().t()
        err_lib = float((ref[sub].float() - exact).norm() / exact.norm())
        t_lib = timeit(lambda: torch.nn.functional.linear(A, B), a.iters)
        fl = 2.0 * M * N * K
        combos = [(int(x), int(y), st) for x in a.variants.split(",") for y in a.dbg.split(",")
                  for st in (a.stagger.split(",") if int(x) == 12 else ["1:-1"])]
        for v, d, st in combos:
            native._K.gemm_set_variant(v)
            native._K.gemm_set_dbg(d)
            native._K.gemm_set_stagger(*[int(t) for t in st.split(":")])
            ours = native.gemm_nt(A, B)
            err = float((ours[sub].float() - exact).norm() / exact.norm())
            t_ours = timeit(lambda: native.gemm_nt(A, B), a.iters)
            native._K.gemm_set_dbg(0)
            row = {"shape": name, "variant": v, "dbg": d, "stagger": st, "M": M, "N": N, "K": K,
                   "ours_us": round(t_ours * 1e6, 1), "hipblaslt_us": round(t_lib * 1e6, 1),
                   "ours_tflops": round(fl / t_ours / 1e12, 1),
                   "hipblaslt_tflops": round(fl / t_lib / 1e12, 1),
                   "speedup": round(t_lib / t_ours, 3), "rel_err": round(err, 5),
                   "rel_err_hipblaslt": round(err_lib, 5)}
            rows.append(row)
            print(json.dumps(row), flush=True)
        native._K.gemm_set_variant(-1)
        native._K.gemm_set_stagger(1, -1)
        del A, B, ours, ref
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
