"""BERT dense-layer weight gradients dW[o, i] = dY^T X over T tokens (fp32 out): the library
path (_Dense: token-split batched hipBLASLt + deterministic slab sum, or one addmm) against the
native TN conv weight-gradient kernel (_NativeDense: conv2d_wgrad, fp32 straight into the
buffer).  Accuracy vs an fp32 reference and HIP-event time per call.

    python tools/dense_wgrad_bench.py [--iters 20]
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
SHAPES = [("qkv", T, 2304, 768), ("attn_out", T, 768, 768), ("ffn1", T, 3072, 768),
          ("ffn2", T, 768, 3072), ("mlm_transform", 10240, 768, 768),
          ("mlm_decoder", 10240, 30528, 768)]


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


def library(dy, x, out):
    T_, o = dy.shape
    i = x.shape[1]
    S = native._wgrad_splits(T_, o, i)
    if S == 1:
        torch.addmm(out, dy.t(), x, out_dtype=torch.float32, out=out)
        return
    part = torch.bmm(dy.view(S, T_ // S, o).transpose(1, 2), x.view(S, T_ // S, i),
                     out_dtype=torch.float32)
    native._K.slab_reduce(part.data_ptr(), out.data_ptr(), o * i, S, 1, native._st())


def ours(dy, x, out):
    T_, o = dy.shape
    i = x.shape[1]
    native.conv2d_wgrad(x.view(T_, 1, 1, i), dy.view(T_, 1, 1, o), (o, 1, 1, i), 1, 0,
                        out=out.view(o, 1, 1, i))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for name, T_, o, i in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(T_, i, device="cuda", generator=g).bfloat16()
        dy = (torch.randn(T_, o, device="cuda", generator=g) / T_ ** 0.5).bfloat16()
        ref = dy.float().t() @ x.float()
        errs = {}
        for nm, fn in (("library", library), ("ours", ours)):
            out = torch.zeros(o, i, device="cuda")
            fn(dy, x, out)
            errs[nm] = float((out - ref).norm() / ref.norm())
        o1 = torch.zeros(o, i, device="cuda")
        t_lib = timeit(lambda: library(dy, x, o1), a.iters)
        t_ours = timeit(lambda: ours(dy, x, o1), a.iters)
        fl = 2.0 * T_ * o * i
        row = {"shape": name, "T": T_, "o": o, "i": i, "library_us": round(t_lib * 1e6, 1),
               "ours_us": round(t_ours * 1e6, 1), "library_tflops": round(fl / t_lib / 1e12, 1),
               "ours_tflops": round(fl / t_ours / 1e12, 1), "speedup": round(t_lib / t_ours, 3),
               "rel_err_library": round(errs["library"], 6), "rel_err_ours": round(errs["ours"], 6)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del x, dy, ref
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
