"""Where a 3x3 conv loses against the GEMM ceiling: for each ResNet-50 3x3 stride-1 shape, time
(batch --batch) the conv forward with / without its BatchNorm-statistics epilogue, the stride-1
data gradient, and a DENSE GEMM of the same M x N x K (random A [M, 9C], B [K, 9C]) on the same
persistent kernel, with / without statistics.  The dense rows are the ceiling the implicit-GEMM
gather could reach; the gap between the two is the gather's cost.

    python tools/conv_gap.py [--batch 1984] [--iters 10]
"""
import argparse
import json

import torch

from distributedtensorflow_amd.ops import native


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
    ap.add_argument("--batch", type=int, default=1984)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    K_ = native.kernels()
    dev = "cuda"
    for name, H, C in (("s1b1c2", 28, 128), ("s2b1c2", 14, 256), ("s3b1c2", 7, 512)):
        B = a.batch
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device=dev) * 0.02).to(torch.bfloat16)
        M = B * H * H
        flop = 2.0 * M * C * 9 * C
        rows = K_.conv_tile_rows([B, H, H, C, H, H, 1, 1, C, 9 * C, H, H, 1, 1, 0, 0, 0],
                                 [r - 1 for r in range(3) for _ in range(3)],
                                 [s - 1 for _ in range(3) for s in range(3)], 0)
        ws = torch.empty(K_.bn_workspace_floats_g(rows, C), device=dev, dtype=torch.float32)
        rec = {"layer": name, "M": M, "N": C, "K": 9 * C}
        rec["conv_fwd_stats_us"] = timeit(lambda: native.conv2d_forward(x, w, 1, 1, stats=ws), a.iters)
        rec["conv_fwd_us"] = timeit(lambda: native.conv2d_forward(x, w, 1, 1), a.iters)
        rec["conv_dgrad_us"] = timeit(
            lambda: native.conv2d_dgrad(x, w, x.shape, 1, 1), a.iters)
        del x
        A = torch.randn(M, 9 * C, device=dev).to(torch.bfloat16)
        Bm = (torch.randn(C, 9 * C, device=dev) * 0.02).to(torch.bfloat16)
        G = K_.gemm_tile_rows(M)
        ws2 = torch.empty(K_.bn_workspace_floats_g(G, C), device=dev, dtype=torch.float32)
        rec["dense_us"] = timeit(lambda: native.gemm_nt(A, Bm), a.iters)
        rec["dense_stats_us"] = timeit(lambda: native.gemm_nt(A, Bm, stats=ws2), a.iters)
        for k in list(rec):
            if k.endswith("_us"):
                rec[k] = round(rec[k], 1)
                rec[k[:-3] + "_tf"] = round(flop / rec[k] * 1e-6, 1)
        print(json.dumps(rec), flush=True)
        del A, Bm
        torch.cuda.empty_cache()
    # stride-2 3x3 data gradients: the phase classes launched one by one vs grouped (classes
    # interleaved per tile; only taken without the BN-backward sums, ops/native.py conv2d_dgrad)
    for name, H, C in (("s1b0c2", 56, 128), ("s2b0c2", 28, 256), ("s3b0c2", 14, 512)):
        B = a.batch
        dy = torch.randn(B, H // 2, H // 2, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device=dev) * 0.02).to(torch.bfloat16)
        rec = {"layer": name + "_dgrad"}
        # with the fused BN-backward sums of the BatchNorm(+ReLU) whose output x is (mkind 2)
        xb = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        st = tuple(torch.rand(C, device=dev) + 0.5 for _ in range(4))
        for tag, grouped in (("split", False), ("grouped", True)):
            native._DGRAD_GROUPED = grouped
            rec[tag + "_us"] = round(timeit(
                lambda: native.conv2d_dgrad(dy, w, (B, H, H, C), 2, 1), a.iters), 1)
            rec[tag + "_bnb_us"] = round(timeit(
                lambda: native.conv2d_dgrad(dy, w, (B, H, H, C), 2, 1,
                                            bnb=(xb, st, None, True, False, None)), a.iters), 1)
        del xb
        native._DGRAD_GROUPED = True
        print(json.dumps(rec), flush=True)
        del dy
        torch.cuda.empty_cache()
    # strided data gradients on the GEMM (output channels >= 256): the persistent kernel with its
    # row-table epilogue vs the round-5 ping-pong kernel
    for name, H, C, K, R in (("s2b0c2", 28, 256, 256, 3), ("s3b0c2", 14, 512, 512, 3),
                             ("s1b0proj", 56, 256, 512, 1), ("s2b0proj", 28, 512, 1024, 1),
                             ("s3b0proj", 14, 1024, 2048, 1)):
        B = a.batch
        dy = torch.randn(B, H // 2, H // 2, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, R, R, C, device=dev) * 0.02).to(torch.bfloat16)
        rec = {"layer": name + "_dgrad_gemm"}
        for tag, on in (("pp2", 1), ("pingpong", 0)):
            K_.gemm_set_pp2_strided(on)
            rec[tag + "_us"] = round(timeit(
                lambda: native.conv2d_dgrad(dy, w, (B, H, H, C), 2, R // 2), a.iters), 1)
        K_.gemm_set_pp2_strided(1)
        print(json.dumps(rec), flush=True)
        del dy
        torch.cuda.empty_cache()
    # projection shortcuts: 1x1 stride 2 forward with the BN statistics epilogue
    for name, H, C, K in (("s1b0proj", 56, 256, 512), ("s2b0proj", 28, 512, 1024),
                          ("s3b0proj", 14, 1024, 2048)):
        B = a.batch
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, 1, 1, C, device=dev) * 0.02).to(torch.bfloat16)
        P = H // 2
        rows = K_.conv_tile_rows([B, H, H, C, P, P, 2, 2, K, C, P, P, 1, 1, 0, 0, 0], [0], [0], 0)
        ws = torch.empty(K_.bn_workspace_floats_g(rows, K), device=dev, dtype=torch.float32)
        us = timeit(lambda: native.conv2d_forward(x, w, 2, 0, stats=ws), a.iters)
        byts = 2.0 * B * P * P * (C + K)
        print(json.dumps({"layer": name, "conv_fwd_stats_us": round(us, 1),
                          "tf": round(2.0 * B * P * P * C * K / us * 1e-6, 1),
                          "tbps": round(byts / us * 1e-6, 2), "tile_rows": rows}), flush=True)
        del x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
