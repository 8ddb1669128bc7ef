"""Per-tile fixed cost of the MFMA GEMM (csrc/kernels/gemm.hip): time C = A . B^T at fixed M, N
over a sweep of K and fit  t = t_fixed + t_step * (K / 64)  per tile round; with
``gemm_set_dbg(1)`` the epilogue (staging, bias/stats, C stores) is skipped, which splits the
fixed cost into prologue and epilogue.  Findings (persistent kernel, register
epilogues): profiles/measurements/r2_gemm_epilogue_probes.jsonl.

    python tools/gemm_overhead.py [--out overhead.jsonl]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributedtensorflow_amd.ops import native  # noqa: E402


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
    ap.add_argument("--out", default=None)
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--N", default="768,2304")
    ap.add_argument("--K", default="64,128,256,512,768,1536,3072")
    ap.add_argument("--variants", default="-1")
    ap.add_argument("--nt", default="0", help="gemm_set_nt values (non-temporal C stores)")
    ap.add_argument("--dbg", default="0,1", help="gemm_set_dbg values: 1 = skip the epilogue")
    a = ap.parse_args()
    rows = []
    for N in [int(x) for x in a.N.split(",")]:
        for v, nt in [(int(v), int(t)) for v in a.variants.split(",") for t in a.nt.split(",")]:
            native._K.gemm_set_variant(v)
            native._K.gemm_set_nt(nt)
            for dbg in [int(x) for x in a.dbg.split(",")]:
                native._K.gemm_set_dbg(dbg)
                ks, ts = [], []
                for K in [int(x) for x in a.K.split(",")]:
                    A = torch.randn(a.M, K, device="cuda").bfloat16()
                    B = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
                    t = timeit(lambda: native.gemm_nt(A, B), a.iters)
                    tiles = -(-a.M // 256) * -(-N // 256)
                    rounds = tiles / 256.0          # tile rounds over 256 CUs
                    row = {"M": a.M, "N": N, "K": K, "variant": v, "nt": nt,
                           "skip_epilogue": dbg,
                           "us": round(t * 1e6, 1), "us_per_round": round(t * 1e6 / rounds, 2),
                           "tflops": round(2.0 * a.M * N * K / t / 1e12, 1)}
                    rows.append(row)
                    print(json.dumps(row), flush=True)
                    ks.append(K / 64)
                    ts.append(t * 1e6 / rounds)
                    del A, B
                slope, icpt = np.polyfit(ks, ts, 1)
                fit = {"fit": True, "N": N, "variant": v, "nt": nt,
                       "skip_epilogue": dbg,
                       "us_per_kstep": round(float(slope), 3),
                       "us_fixed_per_tile": round(float(icpt), 3),
                       "fixed_in_ksteps": round(float(icpt / slope), 2)}
                rows.append(fit)
                print(json.dumps(fit), flush=True)
    native._K.gemm_set_dbg(0)
    native._K.gemm_set_variant(-1)
    native._K.gemm_set_nt(0)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
