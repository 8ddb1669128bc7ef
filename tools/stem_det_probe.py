"""Locate the stem-gradient non-determinism under DTF_WGRAD_SIDE=1: record the stem weight
gradient's inputs (x, dy) and output per backward pass and compare them across passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import resnet50
    from distributedtensorflow_amd.ops import native
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import MirroredStrategy
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    torch.manual_seed(0)
    strat = MirroredStrategy()
    with strat.scope():
        model = resnet50()
        opt = MomentumOptimizer(0.1, 0.9)
        opt.build(list(model.parameters()))
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(B, 224, 224, 3, device="cuda", generator=g).to(torch.bfloat16)
    y = torch.randint(0, 1000, (B,), device="cuda", generator=g)
    rec = []
    orig = native.conv2d_wgrad

    def spy(xb, dy, w_shape, stride, padding, out=None):
        r = orig(xb, dy, w_shape, stride, padding, out=out)
        if xb.shape[-1] == 16:
            torch.cuda.current_stream().synchronize()
            rec[-1].append((xb.detach().clone(), dy.detach().clone(), r.detach().clone()))
        return r
    native.conv2d_wgrad = spy
    grads = []
    for _ in range(4):
        rec.append([])
        out = model(x)
        loss = ops.sparse_softmax_cross_entropy(out, y)
        opt.compute_gradients(loss, list(model.parameters()))
        torch.cuda.synchronize()
        grads.append(opt.space.grad.detach().clone())
    names = [n for n, p in model.named_parameters()]
    for k in range(1, 4):
        a, b = rec[0][0], rec[k][0]
        print(f"pass {k}: stem x same {torch.equal(a[0], b[0])} dy same {torch.equal(a[1], b[1])} "
              f"dW same {torch.equal(a[2], b[2])} flat grads same {torch.equal(grads[0], grads[k])}")
        if not torch.equal(a[1], b[1]):
            d = (a[1].float() - b[1].float()).abs()
            idx = (d > 0).nonzero()
            print("   dy differs at", idx.shape[0], "elements; first", idx[:3].tolist(),
                  "max", float(d.max()))


if __name__ == "__main__":
    main()
