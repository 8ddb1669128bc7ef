"""Grid-cap sweep of the stem's fused max-pool + BN backward passes (reduce / apply) at the
ResNet-50 b1984 stem shape (112 x 112 x 64 -> 56 x 56): microseconds per call per cap."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributedtensorflow_amd.ops import native  # noqa: E402

K = native._K
N, H, W, C = int(sys.argv[1]) if len(sys.argv) > 1 else 1984, 112, 112, 64
P, Q = 56, 56
g = torch.Generator(device="cuda").manual_seed(0)
dy = torch.randn(N, P, Q, C, device="cuda", generator=g).bfloat16()
arg = torch.randint(0, 9, (N, P, Q, C), device="cuda", dtype=torch.uint8, generator=g)
x = torch.randn(N, H, W, C, device="cuda", generator=g).bfloat16()
vec = [torch.rand(C, device="cuda", generator=g) + 0.5 for _ in range(5)]
dx = torch.empty_like(x)
st = torch.cuda.current_stream().cuda_stream


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for cap in (512, 768, 1024, 1536, 2048, 3072, 4096):
    K.pool_bn_bwd_set_caps(cap, cap)
    G = K.pool_bn_bwd_blocks(N, H, W, C)
    part = torch.empty(G * 2 * C, device="cuda")
    red = timeit(lambda: K.pool_bn_bwd_reduce(dy.data_ptr(), arg.data_ptr(), x.data_ptr(),
                                              vec[0].data_ptr(), vec[1].data_ptr(),
                                              vec[3].data_ptr(), vec[4].data_ptr(),
                                              part.data_ptr(), N, H, W, C, P, Q, st))
    app = timeit(lambda: K.pool_bn_bwd_apply(dy.data_ptr(), arg.data_ptr(), x.data_ptr(),
                                             vec[0].data_ptr(), vec[1].data_ptr(),
                                             vec[2].data_ptr(), vec[3].data_ptr(),
                                             vec[4].data_ptr(), dx.data_ptr(), N, H, W, C, P, Q,
                                             st))
    print(json.dumps({"cap": cap, "reduce_us": round(red, 1), "apply_us": round(app, 1)}),
          flush=True)
K.pool_bn_bwd_set_caps(4096, 4096)
