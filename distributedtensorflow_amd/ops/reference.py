"""PyTorch reference implementations of every op in :mod:`distributedtensorflow_amd.ops`.

These are the *oracles* the HIP kernels are tested against and the CPU execution path
(``OneDeviceStrategy("/cpu:0")``, BASELINE config 1).  All image tensors are NHWC
(TF ``channels_last``, the tf.layers default used by the reference CNN,
``run_mnist_distributed.py:50-69``).  Filters are stored ``[K, R, S, C]`` (output channel
major, reduction axis contiguous) which is the layout the MFMA implicit-GEMM kernels consume;
the checkpoint layer converts to TF's ``HWIO`` on save/load.

Math follows the TF1 kernels the reference calls:
  * ``sparse_softmax_cross_entropy`` = mean over the batch (``run_mnist_distributed.py:113``);
  * batch-norm uses biased batch variance for normalisation and the Bessel-corrected
    variance for the moving average (TF ``FusedBatchNorm`` training semantics).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def conv_out_size(h, r, stride, pad_lo, pad_hi):
    return (h + pad_lo + pad_hi - r) // stride + 1


def resolve_padding(padding, h, w, r, s, stride):
    """Return (pad_top, pad_bottom, pad_left, pad_right) for TF-style or explicit padding."""
    sh, sw = _pair(stride)
    if isinstance(padding, str):
        p = padding.upper()
        if p == "VALID":
            return 0, 0, 0, 0
        if p == "SAME":
            oh = -(-h // sh)
            ow = -(-w // sw)
            th = max((oh - 1) * sh + r - h, 0)
            tw = max((ow - 1) * sw + s - w, 0)
            return th // 2, th - th // 2, tw // 2, tw - tw // 2
        raise ValueError(f"unknown padding {padding!r}")
    ph, pw = _pair(padding)
    return ph, ph, pw, pw


def conv2d(x, w, stride=1, padding=0, bias=None):
    """x: [N,H,W,C]; w: [K,R,S,C] -> y: [N,P,Q,K]."""
    n, h, wd, c = x.shape
    k, r, s, c2 = w.shape
    assert c == c2, (x.shape, w.shape)
    pt, pb, pl, pr = resolve_padding(padding, h, wd, r, s, stride)
    xn = x.permute(0, 3, 1, 2)
    if (pt, pl) != (pb, pr):
        xn = F.pad(xn, (pl, pr, pt, pb))
        pad = 0
    else:
        pad = (pt, pl)
    y = F.conv2d(xn, w.to(x.dtype).permute(0, 3, 1, 2), bias, _pair(stride), pad)
    return y.permute(0, 2, 3, 1)


def batch_norm(x, gamma, beta, running_mean=None, running_var=None, training=True,
               momentum=0.997, eps=1e-5, relu=False, residual=None):
    """Fused BN (+ residual add) (+ ReLU) over the channel (last) axis of an NHWC tensor.

    ``momentum`` is TF's *decay*: moving = moving * momentum + batch * (1 - momentum).
    """
    c = x.shape[-1]
    xf = x.float().reshape(-1, c)
    if training:
        mean = xf.mean(0)
        var = xf.var(0, unbiased=False)
        if running_mean is not None:
            n = xf.shape[0]
            with torch.no_grad():
                running_mean.mul_(momentum).add_(mean.detach() * (1 - momentum))
                unb = var.detach() * (n / max(n - 1, 1))
                running_var.mul_(momentum).add_(unb * (1 - momentum))
    else:
        mean, var = running_mean, running_var
    y = (xf - mean) * torch.rsqrt(var + eps) * gamma.float() + beta.float()
    if residual is not None:
        y = y + residual.float().reshape(-1, c)
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype).reshape(x.shape)


def relu(x):
    return torch.relu(x)


def max_pool2d(x, kernel=2, stride=2, padding=0):
    kh, kw = _pair(kernel)
    n, h, w, c = x.shape
    pt, pb, pl, pr = resolve_padding(padding, h, w, kh, kw, stride)
    xn = x.permute(0, 3, 1, 2)
    if (pt, pl) != (pb, pr):
        xn = F.pad(xn, (pl, pr, pt, pb), value=float("-inf"))
        pad = 0
    else:
        pad = (pt, pl)
    y = F.max_pool2d(xn, (kh, kw), _pair(stride), pad)
    return y.permute(0, 2, 3, 1)


def global_avg_pool(x):
    """[N,H,W,C] -> [N,C] (mean over H, W; computed in fp32)."""
    return x.float().mean(dim=(1, 2)).to(x.dtype)


def dense(x, w, b=None, relu=False):
    """x: [M, in]; w: [out, in] (GEMM 'NT' layout); b: [out]."""
    y = F.linear(x, w.to(x.dtype), None if b is None else b.to(x.dtype))
    return torch.relu(y) if relu else y


def sparse_softmax_cross_entropy(logits, labels):
    """Mean over batch of -log softmax(logits)[label] (TF default reduction)."""
    return F.cross_entropy(logits.float(), labels.long())


def softmax_cross_entropy_clipped_sum(logits, onehot):
    """The MLP template's loss: -sum(y * log(clip(softmax(logits), 1e-10, 1)))
    (``templates/00_mnist_replica.py:162-164``)."""
    p = torch.softmax(logits.float(), dim=-1).clamp(1e-10, 1.0)
    return -(onehot.float() * torch.log(p)).sum()


def layer_norm(x, gamma, beta, eps=1e-12):
    return F.layer_norm(x.float(), (x.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


def gelu(x):
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def attention(q, k, v, mask=None, scale=None):
    """q,k,v: [B, H, S, D] -> [B, H, S, D].  mask: additive [B,1,1,S] or None."""
    d = q.shape[-1]
    scale = scale if scale is not None else d ** -0.5
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask.float()
    p = torch.softmax(s, dim=-1)
    return torch.matmul(p, v.float()).to(q.dtype)


def dropout(x, p, training=True):
    return F.dropout(x, p, training)
