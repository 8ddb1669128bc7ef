"""BERT attention kernels (csrc/kernels/nlp.hip) at the BERT-base b512 shape: time per call of
the forward and the backward (delta + dK/dV + dQ), with and without attention dropout, and the
max error of the dropout-free path against an fp32 PyTorch reference on a slice of the batch.

    python tools/attn_bench.py [--batch 512] [--seq 128] [--heads 12] [--iters 20]
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
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    B, S, H, D = a.batch, a.seq, a.heads, 64
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = (torch.randn(B * S, 3 * H * D, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    mask = torch.zeros(B, S, device=dev)
    mask[:, S - 8:] = -10000.0
    do = torch.randn(B * S, H * D, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(B * S, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, S, device=dev)
    delta = torch.empty_like(lse)
    dqkv = torch.empty_like(qkv)
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    scale = D ** -0.5
    flops_f = 4.0 * B * H * S * S * D
    # dropout runs with and without the forward's stored keep decisions (attn_keep_words)
    for p, use_keep in ((0.0, False), (0.1, False), (0.1, True)):
        nk = _K.attn_keep_words(B, S, H, p) if use_keep else 0
        if use_keep and not nk:
            continue
        keep = torch.empty(max(nk, 1), device=dev, dtype=torch.int32)
        kp = keep.data_ptr() if nk else 0
        fwd = lambda: _K.attn_fwd(qkv.data_ptr(), mask.data_ptr(), out.data_ptr(), lse.data_ptr(),  # noqa: E731
                                  B, S, H, scale, p, 1234, st(), kp)
        bwd = lambda: _K.attn_bwd(qkv.data_ptr(), mask.data_ptr(), out.data_ptr(), do.data_ptr(),  # noqa: E731
                                  lse.data_ptr(), delta.data_ptr(), dqkv.data_ptr(), B, S, H,
                                  scale, p, 1234, st(), 0, kp)
        tf = timeit(fwd, a.iters)
        tb = timeit(bwd, a.iters)
        if p > 0.0:
            # same keep decisions either way: the backward's outputs are bit-identical
            fwd()
            bwd()
            torch.cuda.synchronize()
            if not use_keep:
                ref_dqkv = dqkv.clone()
        rec = {"probe": "attn", "B": B, "S": S, "H": H, "dropout": p, "keep_bits": use_keep,
               "fwd_ms": round(tf, 4),
               "bwd_ms": round(tb, 4), "fwd_tflops": round(flops_f / tf / 1e9, 1),
               "bwd_tflops": round(2.5 * flops_f / tb / 1e9, 1)}
        if p == 0.0:
            # fp32 reference on the first 8 sequences
            n = 8
            q3 = qkv[: n * S].float().view(n, S, 3, H, D)
            q, k, v = (q3[:, :, i].permute(0, 2, 1, 3).requires_grad_(True) for i in range(3))
            s = (q @ k.transpose(-1, -2)) * scale + mask[:n, None, None, :]
            o = torch.softmax(s, -1) @ v
            o2 = o.permute(0, 2, 1, 3).reshape(n * S, H * D)
            o2.backward(do[: n * S].float())
            rec["fwd_max_err"] = float((out[: n * S].float() - o2.detach()).abs().max())
            dq3 = dqkv[: n * S].float().view(n, S, 3, H, D)
            for i, t in enumerate((q, k, v)):
                ref = t.grad.permute(0, 2, 1, 3)
                rec["d%s_max_rel" % "qkv"[i]] = float((dq3[:, :, i] - ref).abs().max()
                                                       / ref.abs().max())
        if use_keep:
            rec["dqkv_bit_identical_to_rehash"] = bool(torch.equal(dqkv, ref_dqkv))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
