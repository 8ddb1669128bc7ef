"""A/B of the ping-pong wgrad's 5-slot 32-pixel ring (DEEP) against the 2 x 64-pixel double
buffer: BERT-base dense dW (dense form) and ResNet-50 b1984 multi-tap layers (general form).
One JSON line per shape: microseconds and bitwise equality; plus the L2-resident probe."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from distributedtensorflow_amd.ops import native  # noqa: E402
from wgrad_dense_ab import timeit  # noqa: E402

CASES = [  # name, N, H, W, C, Kout, R, stride, pad
    ("bert_qkv", 65536, 1, 1, 768, 2304, 1, 1, 0),
    ("bert_attn_out", 65536, 1, 1, 768, 768, 1, 1, 0),
    ("bert_ffn1", 65536, 1, 1, 768, 3072, 1, 1, 0),
    ("bert_ffn2", 65536, 1, 1, 3072, 768, 1, 1, 0),
    ("rn50_s2_c3", 1984, 14, 14, 256, 1024, 1, 1, 0),
    ("rn50_s2_c2_3x3", 1984, 14, 14, 256, 256, 3, 1, 1),
    ("rn50_s2b0_c2_3x3_s2", 1984, 28, 28, 256, 256, 3, 2, 1),
    ("rn50_s3_c2_3x3", 1984, 7, 7, 512, 512, 3, 1, 1),
    ("rn50_s3b0_proj_s2", 1984, 14, 14, 1024, 2048, 1, 2, 0),
]


def main():
    out = open(sys.argv[1], "a") if len(sys.argv) > 1 else None
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, N, H, W, C, K, R, st, pad in CASES:
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        x = torch.randn(N, H, W, C, device="cuda", generator=g).bfloat16()
        dy = (torch.randn(N, P, Q, K, device="cuda", generator=g) / (N * P * Q) ** 0.5).bfloat16()
        dw = torch.zeros(K, R, R, C, device="cuda")
        rec = {"shape": name}
        ws = {}
        for deep in (0, 1, 2):
            native._K.wgrad_set_deep(deep)
            us = timeit(lambda: native.conv2d_wgrad(x, dy, (K, R, R, C), st, pad, out=dw))
            rec[f"deep{deep}_us"] = round(us, 1)
            rec[f"deep{deep}_tflops"] = round(2.0 * N * P * Q * K * R * R * C / us / 1e6, 1)
            ws[deep] = native.conv2d_wgrad(x, dy, (K, R, R, C), st, pad).clone()
            if R == 1 and st == 1:
                native._K.wgrad_set_dense(3)
                us = timeit(lambda: native.conv2d_wgrad(x, dy, (K, R, R, C), st, pad, out=dw))
                rec[f"deep{deep}_l2probe_us"] = round(us, 1)
                native._K.wgrad_set_dense(1)
        native._K.wgrad_set_deep(0)
        rec["bit_identical"] = bool(torch.equal(ws[0], ws[1]) and torch.equal(ws[0], ws[2]))
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
        del x, dy, dw, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
