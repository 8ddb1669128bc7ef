"""One dense weight-gradient shape on the TN wgrad kernel, a few calls (a PMC / trace target)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributedtensorflow_amd.ops import native  # noqa: E402

T, o, i = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (65536, 2304, 768))]
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(T, i, device="cuda", generator=g).bfloat16()
dy = (torch.randn(T, o, device="cuda", generator=g) / T ** 0.5).bfloat16()
out = torch.zeros(o, 1, 1, i, device="cuda")
for _ in range(3):
    native.conv2d_wgrad(x.view(T, 1, 1, i), dy.view(T, 1, 1, o), (o, 1, 1, i), 1, 0, out=out)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    native.conv2d_wgrad(x.view(T, 1, 1, i), dy.view(T, 1, 1, o), (o, 1, 1, i), 1, 0, out=out)
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) / 10 * 1e3
print({"T": T, "o": o, "i": i, "us": round(us, 1), "tflops": round(2 * T * o * i / us / 1e6, 1)})
