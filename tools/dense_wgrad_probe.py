"""Probe: BERT-base dense-layer weight gradients dW[o,i] = dY^T X over T = 16384 tokens, fp32
result accumulated into the flat gradient buffer.  hipBLASLt variants (bf16 out + cast + add,
fp32 out_dtype, in-place addmm, split-K bmm) vs the implicit-GEMM wgrad kernel (1x1 conv view)."""
import json

import torch

from distributedtensorflow_amd.ops import native


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1e3, 1)


def main():
    T = 16384
    for o, i in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
        dy = torch.randn(T, o, device="cuda").bfloat16()
        x = torch.randn(T, i, device="cuda").bfloat16()
        tgt = torch.zeros(o, i, device="cuda")
        ref = dy.float().t() @ x.float()
        r = {"o": o, "i": i, "T": T, "gflop": round(2 * T * o * i / 1e9, 1)}
        r["bf16_mm_cast_add"] = timeit(lambda: tgt.add_(torch.mm(dy.t(), x).float()))
        r["mm_out_fp32_add"] = timeit(lambda: tgt.add_(torch.mm(dy.t(), x, out_dtype=torch.float32)))
        try:
            r["addmm_inplace"] = timeit(lambda: torch.addmm(tgt, dy.t(), x, out_dtype=torch.float32, out=tgt))
        except Exception as e:  # noqa: BLE001
            r["addmm_inplace"] = f"err {type(e).__name__}: {str(e)[:80]}"
        for S in (2, 4, 8):
            try:
                r[f"bmm_split{S}"] = timeit(lambda: tgt.add_(torch.bmm(
                    dy.view(S, T // S, o).transpose(1, 2), x.view(S, T // S, i),
                    out_dtype=torch.float32).sum(0)))
            except Exception as e:  # noqa: BLE001
                r[f"bmm_split{S}"] = f"err {type(e).__name__}: {str(e)[:80]}"
        x4, dy4 = x.view(1, 1, T, i), dy.view(1, 1, T, o)
        t4 = tgt.view(o, 1, 1, i)
        r["dtf_wgrad_kernel"] = timeit(lambda: native.conv2d_wgrad(x4, dy4, (o, 1, 1, i), 1, 0, out=t4))
        tgt.zero_()
        native.conv2d_wgrad(x4, dy4, (o, 1, 1, i), 1, 0, out=t4)
        r["err_dtf"] = ((tgt - ref).norm() / ref.norm()).item()
        tgt.zero_()
        torch.addmm(tgt, dy.t(), x, out_dtype=torch.float32, out=tgt)
        r["err_addmm"] = ((tgt - ref).norm() / ref.norm()).item()
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
