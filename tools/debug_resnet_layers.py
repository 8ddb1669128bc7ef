"""Per-block relative error of the native ResNet-50 forward vs the fp32 reference graph, and the
loss trajectory of native vs reference training (same init, same data)."""
import sys

import torch

from distributedtensorflow_amd import ops
from distributedtensorflow_amd.models import resnet50
from distributedtensorflow_amd.optimizers import MomentumOptimizer
from distributedtensorflow_amd.parallel import OneDeviceStrategy


def blocks_outputs(m, x):
    outs = []
    hooks = [b.register_forward_hook(lambda mod, i, o: outs.append(o.detach().float()))
             for b in [m.stem] + list(m.blocks)]
    with torch.no_grad():
        m(x)
    for h in hooks:
        h.remove()
    return outs


def layer_report(n):
    torch.manual_seed(0)
    m = resnet50().cuda().train()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(n, 224, 224, 3, device="cuda", generator=g)
    rm = [b.clone() for b in m.buffers()]
    nat = blocks_outputs(m, x.bfloat16())
    for b, r in zip(m.buffers(), rm):
        b.copy_(r)
    ops.set_backend("reference")
    ref = blocks_outputs(m, x)
    ops.set_backend("auto")
    # chaos check: the fp32 reference itself, fed the bf16-rounded input
    for b, r in zip(m.buffers(), rm):
        b.copy_(r)
    ops.set_backend("reference")
    ref2 = blocks_outputs(m, x.bfloat16().float())
    ops.set_backend("auto")
    for i, (a, b, c) in enumerate(zip(nat, ref, ref2)):
        rel = ((a - b).norm() / b.norm()).item()
        rel2 = ((c - b).norm() / b.norm()).item()
        print(f"block {i:2d} shape {tuple(a.shape)} native-vs-fp32 {rel:.4f}   "
              f"fp32(bf16 input)-vs-fp32 {rel2:.4f}", flush=True)


def train_trace(backend, steps, lr):
    torch.manual_seed(0)
    ops.set_backend(backend)
    with OneDeviceStrategy("cuda").scope():
        m = resnet50()
        opt = MomentumOptimizer(lr, 0.9, weight_decay=1e-4)
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(64, 224, 224, 3, device="cuda", generator=g)
        y = torch.randint(0, 1000, (64,), device="cuda", generator=g)
        xin = x.bfloat16() if backend == "auto" else x
        out = []
        for _ in range(steps):
            loss = ops.sparse_softmax_cross_entropy(m(xin), y)
            opt.minimize(loss)
            out.append(round(loss.item(), 3))
    ops.set_backend("auto")
    print(f"{backend} lr={lr}: {out}", flush=True)


if __name__ == "__main__":
    layer_report(int(sys.argv[1]) if len(sys.argv) > 1 else 16)
    for be in ("auto", "reference"):
        train_trace(be, 20, 0.1)
