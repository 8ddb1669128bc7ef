"""Print the ResNet-50 training loss per step on a fixed synthetic batch (direct-grad on/off)."""
import sys

import torch

from distributedtensorflow_amd import ops
from distributedtensorflow_amd.models import resnet50
from distributedtensorflow_amd.ops import native
from distributedtensorflow_amd.optimizers import MomentumOptimizer
from distributedtensorflow_amd.parallel import OneDeviceStrategy
from distributedtensorflow_amd.train import global_step as gs_mod


def run(direct, steps, lr, batch):
    native._DIRECT_GRAD = direct
    gs_mod.reset_global_step()
    torch.manual_seed(0)
    with OneDeviceStrategy("cuda").scope():
        m = resnet50()
        opt = MomentumOptimizer(lr, 0.9, weight_decay=1e-4)
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(batch, 224, 224, 3, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 1000, (batch,), device="cuda", generator=g)
        out = []
        for _ in range(steps):
            loss = ops.sparse_softmax_cross_entropy(m(x), y)
            opt.minimize(loss)
            out.append(round(loss.item(), 3))
    print(f"direct={direct} lr={lr} batch={batch}: {out}", flush=True)


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    for direct in (True, False):
        run(direct, steps, 0.1, 256)
    run(True, steps, 0.01, 256)
