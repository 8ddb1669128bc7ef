"""BERT FFN data gradient with the GELU derivative in our GEMM's epilogue (gemm_nt_gelu_bwd) at
the bench shape: time per call, next to the plain GEMM and hipBLASLt.

    python tools/gelu_gemm_bench.py [--tokens 65536] [--iters 20]
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
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    M, N, K = a.tokens, 3072, 768
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    do = torch.randn(M, K, device="cuda").bfloat16()
    wt = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()     # [i, o]: B rows
    ga = torch.randn(M, N, device="cuda").bfloat16()
    gb = torch.randn(N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    cs = torch.empty(_K.gemm_tile_rows(M), N, device="cuda")
    fn = lambda: _K.gemm_nt_gelu_bwd(do.data_ptr(), wt.data_ptr(), out.data_ptr(), M, N, K,  # noqa: E731
                                     K, K, ga.data_ptr(), gb.data_ptr(), cs.data_ptr(), st())
    for _ in range(2):
        us = timeit(fn, a.iters)
        print(json.dumps({"probe": "gelu_gemm", "M": M, "N": N, "K": K, "us": round(us, 1),
                          "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}), flush=True)
    # the forward FFN GEMM: ours with the bias + GELU epilogue vs hipBLASLt + our bias_gelu pass
    x = torch.randn(M, K, device="cuda").bfloat16()
    z = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    h = torch.empty_like(z)
    fused = timeit(lambda: _K.gemm_nt_bias_gelu(x.data_ptr(), wt.data_ptr(), z.data_ptr(),
                                                h.data_ptr(), M, N, K, K, K, gb.data_ptr(), st()),
                   a.iters)

    def two_pass():
        y = torch.nn.functional.linear(x, wt)
        _K.bias_gelu_fwd(y.data_ptr(), gb.data_ptr(), h.data_ptr(), M, N, st())
    lib2 = timeit(two_pass, a.iters)
    print(json.dumps({"probe": "ffn1_fwd", "fused_bias_gelu_gemm_us": round(fused, 1),
                      "hipblaslt_plus_bias_gelu_us": round(lib2, 1)}), flush=True)
    plain = timeit(lambda: native.gemm_nt(do, wt), a.iters)
    lib = timeit(lambda: torch.nn.functional.linear(do, wt), a.iters)
    print(json.dumps({"probe": "gelu_gemm", "plain_gemm_nt_us": round(plain, 1),
                      "hipblaslt_us": round(lib, 1)}), flush=True)


if __name__ == "__main__":
    main()
