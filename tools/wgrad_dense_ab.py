"""A/B of the ping-pong wgrad kernel's DENSE form (no pixel decode) against its general form and
the library GEMM, on BERT-base's dense weight gradients and ResNet-50's stage-3/4 1x1 convs.
One JSON line per shape: microseconds, TFLOP/s, bitwise equality of the two forms."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributedtensorflow_amd.ops import native  # noqa: E402

SHAPES = [  # name, pixels (tokens), Kout (o), C (i)
    ("bert_qkv", 65536, 2304, 768),
    ("bert_attn_out", 65536, 768, 768),
    ("bert_ffn1", 65536, 3072, 768),
    ("bert_ffn2", 65536, 768, 3072),
    ("rn50_s0_c1_b1984", 1984 * 3136, 64, 256),
    ("rn50_s0_c3_b1984", 1984 * 3136, 256, 64),
    ("rn50_s1_c1_b1984", 1984 * 784, 128, 512),
    ("rn50_s1_c3_b1984", 1984 * 784, 512, 128),
    ("rn50_s2_c1_b1984", 1984 * 196, 256, 1024),
    ("rn50_s2_c3_b1984", 1984 * 196, 1024, 256),
    ("rn50_s3_c1_b1984", 1984 * 49, 512, 2048),
    ("rn50_s3_c3_b1984", 1984 * 49, 2048, 512),
]


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    out = open(sys.argv[1], "a") if len(sys.argv) > 1 else None
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, T, o, i in SHAPES:
        x = torch.randn(T, i, device="cuda", generator=g).bfloat16()
        dy = (torch.randn(T, o, device="cuda", generator=g) / T ** 0.5).bfloat16()
        dw = torch.zeros(o, 1, 1, i, device="cuda")
        xv, dv = x.view(T, 1, 1, i), dy.view(T, 1, 1, o)
        res = {}
        for mode in (0, 1):
            native._K.wgrad_set_dense(mode)
            res[mode] = timeit(lambda: native.conv2d_wgrad(xv, dv, (o, 1, 1, i), 1, 0, out=dw))
            res[f"w{mode}"] = native.conv2d_wgrad(xv, dv, (o, 1, 1, i), 1, 0).clone()
        native._K.wgrad_set_dense(1)
        lib = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        fl = 2.0 * T * o * i
        rec = {"shape": name, "T": T, "o": o, "i": i, "general_us": round(res[0], 1),
               "dense_us": round(res[1], 1), "library_us": round(lib, 1),
               "dense_tflops": round(fl / res[1] / 1e6, 1),
               "general_tflops": round(fl / res[0] / 1e6, 1),
               "library_tflops": round(fl / lib / 1e6, 1),
               "bit_identical": bool(torch.equal(res["w0"], res["w1"]))}
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
        del x, dy, dw, res
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
