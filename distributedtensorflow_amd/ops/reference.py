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


# ----------------------------------------------------------------------------- transformer ops
# Bit-exact twins of csrc/kernels/nlp.hip (same hash-based dropout masks), used as the CPU path
# and as the oracle of the GPU numerics tests.

_M32 = 0xFFFFFFFF


def _fmix32(h):
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def drop_threshold(p):
    import numpy as np
    if p <= 0:
        return 0
    t = float(np.float32(p)) * 4294967296.0
    return 4294967295 if t >= 4294967295.0 else int(t)


def keep_mask(seed, idx, p):
    """keep(idx) of the kernels: fmix32(idx * 0x9E3779B1 + seed) >= p * 2^32 (uint32 math)."""
    idx = idx.to(torch.int64) & _M32
    h = _fmix32((idx * 0x9E3779B1 + int(seed)) & _M32)
    return h >= drop_threshold(p)


def _drop(x, p, seed, idx):
    if p <= 0:
        return x
    return torch.where(keep_mask(seed, idx, p), x / (1.0 - float(torch.tensor(p, dtype=torch.float32))), torch.zeros_like(x))


def _rows_cols_idx(M, H, device):
    return torch.arange(M * H, device=device, dtype=torch.int64).view(M, H)


def _next_seed(p):
    return int(torch.randint(0, 2 ** 31 - 1, (1,), device="cpu").item()) if p > 0 else 0


def _round_st(t, dtype):
    """Round the forward value to ``dtype`` (what the kernels store) while the gradient passes
    through in full precision (the kernels accumulate gradients in fp32)."""
    if dtype == t.dtype:
        return t
    return t + (t.to(dtype).to(t.dtype) - t).detach()


def _ln(s, gamma, beta, eps):
    mean = s.mean(-1, keepdim=True)
    var = s.var(-1, unbiased=False, keepdim=True)
    return (s - mean) * torch.rsqrt(var + eps) * gamma.float() + beta.float()


def bias_dropout_add_layer_norm(a, bias, residual, gamma, beta, p=0.0, training=True, eps=1e-12,
                                seed=None):
    p = p if training else 0.0
    H = a.shape[-1]
    s = a.float().reshape(-1, H)
    if bias is not None:
        s = s + bias.float()
    if p > 0:
        seed = _next_seed(p) if seed is None else seed
        s = _drop(s, p, seed, _rows_cols_idx(s.shape[0], H, s.device))
    if residual is not None:
        s = s + residual.float().reshape(-1, H)
    s = _round_st(s, a.dtype)
    return _ln(s, gamma, beta, eps).to(a.dtype).view(a.shape)


def embedding_layer_norm(ids, token_type_ids, word, pos, typ, gamma, beta, p=0.0, training=True,
                         eps=1e-12, seed=None, dtype=None):
    p = p if training else 0.0
    B, S = ids.shape
    H = word.shape[1]
    dtype = dtype or word.dtype
    tt = token_type_ids if token_type_ids is not None else torch.zeros_like(ids)
    w32, p32, t32 = (_round_st(t.float(), dtype) for t in (word, pos, typ))
    s = (w32[ids] + p32[:S].unsqueeze(0) + t32[tt]).reshape(B * S, H)
    s = _round_st(s, dtype)
    y = _ln(s, gamma, beta, eps)
    if p > 0:
        seed = _next_seed(p) if seed is None else seed
        y = _drop(y, p, seed, _rows_cols_idx(B * S, H, y.device))
    return y.to(dtype)


def bias_gelu(a, bias=None):
    x = a.float() + (bias.float() if bias is not None else 0.0)
    return F.gelu(x, approximate="tanh").to(a.dtype)


def attention_qkv(qkv, mask, batch, seq_len, heads, p=0.0, training=True, scale=None, seed=None):
    """qkv [B*S, 3*H*D] (all q heads | all k heads | all v heads) -> [B*S, H*D]."""
    p = p if training else 0.0
    B, S, Hh = batch, seq_len, heads
    D = qkv.shape[-1] // (3 * Hh)
    scale = D ** -0.5 if scale is None else scale
    x = qkv.float().view(B, S, 3, Hh, D)
    q, k, v = (x[:, :, i].permute(0, 2, 1, 3) for i in range(3))     # [B, H, S, D]
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    if mask is not None:
        s = s + mask.float().view(B, 1, 1, S)
    prob = torch.softmax(s, dim=-1)
    if p > 0:
        seed = _next_seed(p) if seed is None else seed
        idx = torch.arange(B * Hh * S * S, device=qkv.device, dtype=torch.int64).view(B, Hh, S, S)
        prob = _drop(prob, p, seed, idx)
    o = torch.matmul(prob, v)                                         # [B, H, S, D]
    return o.permute(0, 2, 1, 3).reshape(B * S, Hh * D).to(qkv.dtype)


def mlm_loss(logits, labels, weights=None, vocab=None):
    """sum_i w_i * nll_i / sum_i w_i  (google-research/bert run_pretraining.py).  ``vocab``: the
    class count when the logits rows are padded past it (columns from ``vocab`` on are ignored)."""
    if vocab is not None and vocab != logits.shape[-1]:
        logits = logits[..., :vocab]
    nll = F.cross_entropy(logits.float(), labels.reshape(-1).long(), reduction="none")
    if weights is None:
        return nll.mean()
    w = weights.reshape(-1).float()
    return (w * nll).sum() / w.sum().clamp_min(1e-5)


def space_to_depth_operands(x, w, stride, pad, want_x=True):
    """Rewrite a strided conv (the ResNet stem: 7x7 / 2, pad 3, C = 3) as a stride-1 VALID conv
    on the space-to-depth input.  Output pixel p reads padded input rows s*p + r, r < R; with
    r = s*i + a that is row p + i of the s2d image at sub-row a, so

        x' [N, P + R' - 1, Q + S' - 1, s*s*C']  (C' = C zero-padded so s*s*C' % 8 == 0)
        w' [K, R', S', s*s*C']                  (R' = ceil(R / s), taps past R are zero)

    compute exactly the original conv.  For the stem: 16 taps x 16 channels = K 256 of which
    147 are real (vs 49 taps x 8 padded channels = 392), and whole 32-B tap rows per pixel.
    Both rewrites are differentiable torch views/pads (w' keeps autograd back to the master).
    ``want_x=False`` skips x' (returned as None) for callers with a native layout kernel."""
    n, h, wd, c = x.shape
    K, R, S, C = w.shape
    s = stride
    P = (h + 2 * pad - R) // s + 1
    Q = (wd + 2 * pad - S) // s + 1
    Rp, Sp = -(-R // s), -(-S // s)
    cp = c
    while (s * s * cp) % 8:
        cp += 1
    Hn, Wn = s * (P + Rp - 1), s * (Q + Sp - 1)
    wp = torch.nn.functional.pad(w, (0, cp - C, 0, s * Sp - S, 0, s * Rp - R))
    ws = wp.view(K, Rp, s, Sp, s, cp).permute(0, 1, 3, 2, 4, 5).reshape(K, Rp, Sp, s * s * cp)
    if not want_x:
        return None, ws
    xp = torch.nn.functional.pad(x, (0, cp - c, pad, Wn - wd - pad, pad, Hn - h - pad))
    xs = xp.view(n, Hn // s, s, Wn // s, s, cp).permute(0, 1, 3, 2, 4, 5).reshape(
        n, Hn // s, Wn // s, s * s * cp)
    return xs.contiguous(), ws
