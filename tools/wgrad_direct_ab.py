"""A/B of the ping-pong wgrad kernel's pixel decode on ResNet-50's multi-tap / strided layers
(b1984): per-row DIRECT decode (each lane decodes the rows it fetches) against the lane-per-pixel
decode shuffled to the DMA rows.  One JSON line per layer: microseconds and bitwise equality."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributedtensorflow_amd.ops import native  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1984
LAYERS = [  # name, H, W, C, Kout, R, stride, pad
    ("s2_c2_3x3", 14, 14, 256, 256, 3, 1, 1),
    ("s2b0_c2_3x3_s2", 28, 28, 256, 256, 3, 2, 1),
    ("s2b0_proj_1x1_s2", 28, 28, 512, 1024, 1, 2, 0),
    ("s3_c2_3x3", 7, 7, 512, 512, 3, 1, 1),
    ("s3b0_c2_3x3_s2", 14, 14, 512, 512, 3, 2, 1),
    ("s3b0_proj_1x1_s2", 14, 14, 1024, 2048, 1, 2, 0),
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
    for name, H, W, C, K, R, st, pad in LAYERS:
        P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
        x = torch.randn(B, H, W, C, device="cuda", generator=g).bfloat16()
        dy = (torch.randn(B, P, Q, K, device="cuda", generator=g) / (B * P * Q) ** 0.5).bfloat16()
        dw = torch.zeros(K, R, R, C, device="cuda")
        res = {}
        for mode in (0, 1, 2):
            native._K.wgrad_set_direct(mode)
            res[mode] = timeit(lambda: native.conv2d_wgrad(x, dy, (K, R, R, C), st, pad, out=dw))
            res[f"w{mode}"] = native.conv2d_wgrad(x, dy, (K, R, R, C), st, pad).clone()
        native._K.wgrad_set_direct(0)
        fl = 2.0 * B * P * Q * K * R * R * C
        rec = {"layer": name, "batch": B, "shuffle_us": round(res[0], 1),
               "direct_us": round(res[1], 1), "direct_tflops": round(fl / res[1] / 1e6, 1),
               "shuffle_tflops": round(fl / res[0] / 1e6, 1),
               "readlane_us": round(res[2], 1),
               "readlane_tflops": round(fl / res[2] / 1e6, 1),
               "bit_identical": bool(torch.equal(res["w0"], res["w1"]) and
                                     torch.equal(res["w0"], res["w2"]))}
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
        del x, dy, dw, res
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
