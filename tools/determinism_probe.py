"""Run-to-run determinism of the native ResNet-50 step: the same init, data and one
forward+backward twice in one process; report which parameters' gradients differ bit-wise
(and the first differing forward activation), to locate non-deterministic kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import resnet50
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import MirroredStrategy
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    torch.manual_seed(0)
    strat = MirroredStrategy()
    with strat.scope():
        model = resnet50()
        opt = MomentumOptimizer(0.1, 0.9)
        opt.build(list(model.parameters()))
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, S, S, 3, device="cuda", generator=g).to(torch.bfloat16)
    y = torch.randint(0, 1000, (B,), device="cuda", generator=g)
    grads, logits = [], []
    for _ in range(3):
        out = model(x)
        logits.append(out.detach().clone())
        loss = ops.sparse_softmax_cross_entropy(out, y)
        opt.compute_gradients(loss, list(model.parameters()))
        torch.cuda.synchronize()
        grads.append(opt.space.grad.detach().clone())
    print("logits identical:", [torch.equal(logits[0], l) for l in logits[1:]])
    names = {id(p): n for n, p in model.named_parameters()}
    for k in (1, 2):
        bad = []
        for v, o in zip(opt.space.order, opt.space.offsets):
            a, b = grads[0][o:o + v.numel()], grads[k][o:o + v.numel()]
            if not torch.equal(a, b):
                rel = ((a - b).abs().max() / a.abs().max().clamp_min(1e-30)).item()
                bad.append((names.get(id(v)), tuple(v.shape), f"{rel:.2e}"))
        print(f"run {k}: {len(bad)} of {len(opt.space.order)} parameter gradients differ")
        for row in bad[:40]:
            print("  ", row)


if __name__ == "__main__":
    main()
