"""Timing probes of the row-streaming GEMM's plain K = 256 kernel (compile-time variants, so the
measured kernel's own code is unperturbed): 0 full, 1 no MFMAs, 2 no LDS staging of C, 4 no
chunk barrier, 8 C stores out of range, and combinations.

    python tools/stream_probe.py [--M 388864 --N 1024]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributedtensorflow_amd.ops import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=388864)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(a.M, 256, device="cuda", generator=g).bfloat16()
    B = (torch.randn(a.N, 256, device="cuda", generator=g) / 16).bfloat16()
    C = torch.empty(a.M, a.N, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for _ in range(a.rounds):              # interleaved rounds in one process
        for p in (0, 1, 2, 4, 8, 10, 11, 15):
            fn = lambda: native._K.gemm_stream_probe(A.data_ptr(), B.data_ptr(), C.data_ptr(),  # noqa: E731
                                                     a.M, a.N, p, st)
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(p, []).append(s.elapsed_time(e) / a.iters * 1e3)
    for p, v in res.items():
        print(json.dumps({"probe": p, "M": a.M, "N": a.N, "us": [round(x, 1) for x in v],
                          "min_us": round(min(v), 1)}))


if __name__ == "__main__":
    main()
