"""Where does a bottleneck's backward diverge from fp32?  Runs one ResNet-50 block (training
mode) natively and on the fp32 reference graph from the same bf16 input and upstream gradient,
and prints the relative error of the gradient at every conv output / BN output inside it.

    python tools/block_grad_probe.py [--block 0] [--n 16] [--s 96]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtensorflow_amd import ops  # noqa: E402
from distributedtensorflow_amd.models import resnet as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--s", type=int, default=96)
    ap.add_argument("--env", default="")
    a = ap.parse_args()
    torch.manual_seed(0)
    m = R.resnet50().cuda().train()
    with torch.no_grad():
        for mod in m.modules():
            if hasattr(mod, "gamma"):
                mod.gamma.uniform_(0.5, 1.5)
                mod.beta.normal_(0.0, 0.1)
        for p in m.parameters():
            p.copy_(p.bfloat16().float())
    x = torch.randn(a.n, a.s, a.s, 3, device="cuda").bfloat16()
    with torch.no_grad():
        act = m.stem(x, pool=True)
        for b in m.blocks[:a.block]:
            act = b(act)
    blk = m.blocks[a.block]
    grads = {}
    orig = R.ConvBN.forward

    def fwd(self, xx, relu=True, residual=None, residual_to_conv=False, grad_share=None):
        tag = [k for k, v in blk.named_children() if v is self][0]
        y = ops.conv2d(xx, self.conv.kernel, self.conv.strides, self.conv.padding,
                       bn_stats=self.bn.training, grad_share=grad_share)
        if y.requires_grad:
            y.register_hook(lambda g, t=tag: grads.setdefault(mode, {}).__setitem__(t + ".conv_out", g.float()))
        z = self.bn(y, relu=relu, residual=residual, residual_to_conv=residual_to_conv)
        if z.requires_grad:
            z.register_hook(lambda g, t=tag: grads.setdefault(mode, {}).__setitem__(t + ".bn_out", g.float()))
        return z

    R.ConvBN.forward = fwd
    g = None
    saved = [b_.clone() for b_ in blk.buffers()]
    outs = {}
    for mode in ("native", "reference"):
        for b_, s_ in zip(blk.buffers(), saved):
            b_.copy_(s_)
        for p in blk.parameters():
            p.grad = None
        ops.set_backend("reference" if mode == "reference" else "auto")
        xi = (act.float() if mode == "reference" else act).detach().clone().requires_grad_(True)
        y = blk(xi)
        if g is None:
            g = torch.randn(y.shape, device="cuda").bfloat16()
        y.backward(g.to(y.dtype))
        torch.cuda.synchronize()
        outs[mode] = (y.detach().float(), xi.grad.float(),
                      {n: p.grad.float().clone() for n, p in blk.named_parameters()})
    ops.set_backend("auto")
    R.ConvBN.forward = orig
    rel = lambda u, v: ((u - v).norm() / v.norm().clamp_min(1e-12)).item()
    print("fwd", rel(outs["native"][0], outs["reference"][0]))
    print("dx", rel(outs["native"][1], outs["reference"][1]))
    for k in grads["reference"]:
        if k in grads.get("native", {}):
            print("grad at", k, rel(grads["native"][k], grads["reference"][k]))
        else:
            print("grad at", k, "(no native hook)")
    for n in outs["native"][2]:
        print("param", n, rel(outs["native"][2][n], outs["reference"][2][n]))


if __name__ == "__main__":
    main()
