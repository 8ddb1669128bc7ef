"""Where does the persistent GEMM (variant 15) differ from the ping-pong kernel (variant 8)?
Prints, per epilogue mode, the mismatch count and its distribution over tiles / tile rows / tile
columns (a debugging probe for gemm.hip gemm_pp2_kernel)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from distributedtensorflow_amd.ops import native as n  # noqa: E402


def run(v, fn):
    n._K.gemm_set_variant(v)
    try:
        o = fn()
        torch.cuda.synchronize()
        return o
    finally:
        n._K.gemm_set_variant(-1)


def report(name, x, y):
    d = (x != y)
    cnt = int(d.sum())
    print(f"{name}: mismatches {cnt} of {d.numel()}", flush=True)
    if cnt == 0:
        return
    idx = d.nonzero()
    r, c = idx[:, 0], idx[:, 1]
    tiles_n = (x.shape[1] + 255) // 256
    tile = (r // 256) * tiles_n + c // 256
    print("  tiles:", torch.unique(tile)[:40].tolist(), "n_tiles", int(torch.unique(tile).numel()))
    print("  rows%256:", torch.bincount(r % 256, minlength=256).nonzero().flatten()[:64].tolist())
    print("  cols%256:", torch.bincount(c % 256, minlength=256).nonzero().flatten()[:64].tolist())
    k = idx[:5]
    for rr, cc in k.tolist():
        print("   ", rr, cc, float(x[rr, cc]), float(y[rr, cc]))


M, N, K = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 2304, 768))]
g = torch.Generator(device="cuda").manual_seed(M + N + K)
a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
cin = torch.randn(M, N, device="cuda", generator=g).bfloat16()
report("plain", run(15, lambda: n.gemm_nt(a, b)), run(8, lambda: n.gemm_nt(a, b)))
report("cin", run(15, lambda: n.gemm_nt(a, b, cin=cin.clone())),
       run(8, lambda: n.gemm_nt(a, b, cin=cin.clone())))
c15 = run(15, lambda: n.gemm_nt(a, b, cin=cin.clone()))
c15b = run(15, lambda: n.gemm_nt(a, b, cin=cin.clone()))
report("cin run-to-run", c15, c15b)
ref = (a.float() @ b.float().t() + cin.float())
print("cin err v15", float((c15.float() - ref).norm() / ref.norm()))
