"""Timing probe: the ping-pong wgrad's dense form with streamed operands (FORM 1) against the
same launch re-reading one 64-row step from L2 (FORM 3, wrong results) -- how much of the
kernel's time is operand latency rather than the LDS / MFMA schedule."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributedtensorflow_amd.ops import native  # noqa: E402
from wgrad_dense_ab import timeit  # noqa: E402

for name, T, o, i in [("bert_qkv", 65536, 2304, 768), ("bert_ffn1", 65536, 3072, 768),
                      ("bert_ffn2", 65536, 768, 3072), ("rn50_s3_c3_b1984", 1984 * 49, 2048, 512)]:
    x = torch.randn(T, i, device="cuda").bfloat16()
    dy = torch.randn(T, o, device="cuda").bfloat16()
    dw = torch.zeros(o, 1, 1, i, device="cuda")
    xv, dv = x.view(T, 1, 1, i), dy.view(T, 1, 1, o)
    r = {"shape": name}
    for mode in (1, 3):
        native._K.wgrad_set_dense(mode)
        us = timeit(lambda: native.conv2d_wgrad(xv, dv, (o, 1, 1, i), 1, 0, out=dw))
        r[f"form{mode}_us"] = round(us, 1)
        r[f"form{mode}_tflops"] = round(2.0 * T * o * i / us / 1e6, 1)
    native._K.wgrad_set_dense(1)
    print(json.dumps(r), flush=True)
