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
    ap.add_argument("--variants", default="0",
                    help="comma list of gemm.hip pipeline variants to time (gemm_set_variant)")
    a = ap.parse_args()
    rows = []
    for name, M, N, K in SHAPES:
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
        for v in [int(x) for x in a.variants.split(",")]:
            native._K.gemm_set_variant(v)
            ours = native.gemm_nt(A, B)
            err = float((ours[sub].float() - exact).norm() / exact.norm())
            t_ours = timeit(lambda: native.gemm_nt(A, B), a.iters)
            row = {"shape": name, "variant": v, "M": M, "N": N, "K": K,
                   "ours_us": round(t_ours * 1e6, 1), "hipblaslt_us": round(t_lib * 1e6, 1),
                   "ours_tflops": round(fl / t_ours / 1e12, 1),
                   "hipblaslt_tflops": round(fl / t_lib / 1e12, 1),
                   "speedup": round(t_lib / t_ours, 3), "rel_err": round(err, 5),
                   "rel_err_hipblaslt": round(err_lib, 5)}
            rows.append(row)
            print(json.dumps(row), flush=True)
        native._K.gemm_set_variant(-1)
        del A, B, ours, ref
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
