"""fp32 ops on the HIP kernels of ``csrc/kernels/f32.hip`` -- the reference workload at the
reference's own precision (``run_mnist_distributed.py`` trains fp32 end to end; SURVEY.md
K3-K13).  Matrix work runs on the f32-input MFMA (v_mfma_f32_16x16x4_f32, exact fp32 fma-chain
numerics); weight / bias gradients go straight into the optimizer's fp32 flat gradient buffer
(the GEMM epilogue accumulates there).
"""
from __future__ import annotations

import torch

from .native import _K, _direct_grad, _grad_ready, _p, _pair, _st
from .reference import resolve_padding

_F32 = torch.float32


def _check(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or t.dtype != _F32):
            raise TypeError(f"fp32 native op expects CUDA fp32 tensors, got {t.dtype} on {t.device}")


def gemm_f32(M, N, K, a, sam, sak, b, sbn, sbk, c, scm, scn, bias=None, relu=False,
             accumulate=False, alpha=1.0):
    """c[m*scm + n*scn] (+)= act(alpha * sum_k a[m*sam + k*sak] * b[n*sbn + k*sbk] + bias[n]).
    Few output tiles over a long K (weight gradients) run split-K through a slab workspace with
    a deterministic in-order sum."""
    S = _K.gemm_f32_splits(M, N, K)
    ws = torch.empty(S * M * N, device=c.device, dtype=_F32) if S > 1 else None
    _K.gemm_f32(a.data_ptr(), b.data_ptr(), c.data_ptr(), _p(bias), M, N, K, sam, sak, sbn, sbk,
                scm, scn, float(alpha), int(relu), int(accumulate), _p(ws), _st())
    return c


def _bias_relu_bwd(dy, y, b_master, relu, need_b):
    """dz = dy * (y > 0) (when relu) and db = column sums of dz (into the flat buffer when it
    exposes one).  Returns (dz, db_or_None)."""
    T, N = dy.shape
    if not relu and not need_b:
        return dy, None
    dz = torch.empty_like(dy) if relu else dy
    ws = torch.empty(_K.bias_relu_bwd_f32_ws_floats(N), device=dy.device, dtype=_F32)
    tb = _direct_grad(b_master) if need_b else None
    dbuf = (tb if tb is not None else torch.empty(N, device=dy.device, dtype=_F32)) \
        if need_b else None
    _K.bias_relu_bwd_f32(dy.data_ptr(), _p(y) if relu else dy.data_ptr(), dz.data_ptr(), T, N,
                         ws.data_ptr(), _p(dbuf), int(tb is not None), int(relu), _st())
    db = None
    if need_b:
        if tb is not None:
            _grad_ready(b_master)
        else:
            db = dbuf.to(b_master.dtype)
    return dz, db


def _weight_grad(w_master, compute):
    """compute(out, accumulate) writes dW; straight into the flat fp32 grad when possible."""
    target = _direct_grad(w_master)
    if target is not None:
        compute(target, True)
        _grad_ready(w_master)
        return None
    out = torch.empty(w_master.shape, device=w_master.device, dtype=_F32)
    compute(out, False)
    return out.to(w_master.dtype)


class _DenseF32(torch.autograd.Function):
    """fp32 dense: y = act(x W^T + b) (``layout="OI"``, W [out, in]) or act(x W + b)
    (``layout="IO"``, the MLP template's ``tf.nn.xw_plus_b`` weights [in, out])."""

    @staticmethod
    def forward(ctx, x, w, b, relu, layout):
        i = x.shape[-1]
        x2 = x.reshape(-1, i).contiguous()
        M = x2.shape[0]
        o = w.shape[0] if layout == "OI" else w.shape[1]
        wd = w.detach()
        sbn, sbk = (i, 1) if layout == "OI" else (1, o)
        y = torch.empty(M, o, device=x.device, dtype=_F32)
        gemm_f32(M, o, i, x2, i, 1, wd, sbn, sbk, y, o, 1,
                 bias=b.detach().contiguous() if b is not None else None, relu=relu)
        ctx.save_for_backward(x2, wd, y if relu else None)
        ctx.meta = (relu, layout, x.shape, o)
        ctx.params = (w, b)
        return y.view(*x.shape[:-1], o)

    @staticmethod
    def backward(ctx, dy):
        x2, wd, y = ctx.saved_tensors
        relu, layout, xshape, o = ctx.meta
        w, b = ctx.params
        ctx.params = None
        M, i = x2.shape
        dy2 = dy.reshape(M, o).to(_F32).contiguous()
        dz, db = _bias_relu_bwd(dy2, y, b, relu, b is not None and ctx.needs_input_grad[2])
        dw = dx = None
        if ctx.needs_input_grad[1]:
            scm, scn = (i, 1) if layout == "OI" else (1, o)
            dw = _weight_grad(w, lambda out, acc: gemm_f32(o, i, M, dz, 1, o, x2, 1, i, out,
                                                           scm, scn, accumulate=acc))
        if ctx.needs_input_grad[0]:
            sbn, sbk = (1, i) if layout == "OI" else (o, 1)
            dx = torch.empty(M, i, device=dy.device, dtype=_F32)
            gemm_f32(M, i, o, dz, o, 1, wd, sbn, sbk, dx, i, 1)
            dx = dx.view(xshape)
        return dx, dw, db, None, None


def dense(x, w, b=None, relu=False, layout="OI"):
    _check(x, w)
    return _DenseF32.apply(x, w, b, bool(relu), layout)


class _ConvF32(torch.autograd.Function):
    """fp32 conv (+bias)(+ReLU): im2col + f32 MFMA GEMM with the bias/ReLU epilogue; backward
    fused ReluGrad/BiasAddGrad, dW = dz^T cols into the flat buffer, dx = col2im(dz W)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding, relu):
        x = x.contiguous()
        n, h, wd_, c = x.shape
        K, R, S, C = w.shape
        sh, sw = _pair(stride)
        pt, pb, pl, pr = resolve_padding(padding, h, wd_, R, S, stride)
        P = (h + pt + pb - R) // sh + 1
        Q = (wd_ + pl + pr - S) // sw + 1
        M, TC = n * P * Q, R * S * C
        cols = torch.empty(M, TC, device=x.device, dtype=_F32)
        _K.im2col_f32(x.data_ptr(), cols.data_ptr(), n, h, wd_, c, P, Q, sh, sw, R, S, pt, pl,
                      _st())
        wdet = w.detach().contiguous()
        y = torch.empty(M, K, device=x.device, dtype=_F32)
        gemm_f32(M, K, TC, cols, TC, 1, wdet, TC, 1, y, K, 1,
                 bias=b.detach().contiguous() if b is not None else None, relu=relu)
        ctx.save_for_backward(cols, wdet, y if relu else None)
        ctx.meta = (relu, (n, h, wd_, c), (P, Q, sh, sw, R, S, pt, pl))
        ctx.params = (w, b)
        return y.view(n, P, Q, K)

    @staticmethod
    def backward(ctx, dy):
        cols, wdet, y = ctx.saved_tensors
        relu, (n, h, wd_, c), (P, Q, sh, sw, R, S, pt, pl) = ctx.meta
        w, b = ctx.params
        ctx.params = None
        K = wdet.shape[0]
        M, TC = cols.shape
        dy2 = dy.reshape(M, K).to(_F32).contiguous()
        dz, db = _bias_relu_bwd(dy2, y, b, relu, b is not None and ctx.needs_input_grad[2])
        dw = dx = None
        if ctx.needs_input_grad[1]:
            dw = _weight_grad(w, lambda out, acc: gemm_f32(K, TC, M, dz, 1, K, cols, 1, TC, out,
                                                           TC, 1, accumulate=acc))
        if ctx.needs_input_grad[0]:
            dcols = torch.empty(M, TC, device=dy.device, dtype=_F32)
            gemm_f32(M, TC, K, dz, K, 1, wdet, 1, TC, dcols, TC, 1)
            dx = torch.empty(n, h, wd_, c, device=dy.device, dtype=_F32)
            _K.col2im_f32(dcols.data_ptr(), dx.data_ptr(), n, h, wd_, c, P, Q, sh, sw, R, S, pt,
                          pl, _st())
        return dx, dw, db, None, None, None


def conv2d_bias_relu(x, w, b=None, stride=1, padding=0, relu=True):
    _check(x, w)
    return _ConvF32.apply(x, w, b, stride, padding, bool(relu))


def conv2d(x, w, stride=1, padding=0):
    return conv2d_bias_relu(x, w, None, stride, padding, False)


class _MaxPoolF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s):
        x = x.contiguous()
        n, h, w, c = x.shape
        P, Q = (h - k) // s + 1, (w - k) // s + 1
        y = torch.empty(n, P, Q, c, device=x.device, dtype=_F32)
        arg = torch.empty(n, P, Q, c, device=x.device, dtype=torch.uint8)
        _K.maxpool_f32_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), n, h, w, c, P, Q, k, s,
                           _st())
        ctx.save_for_backward(arg)
        ctx.meta = (x.shape, k, s)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        (n, h, w, c), k, s = ctx.meta
        P, Q = arg.shape[1], arg.shape[2]
        dy = dy.to(_F32).contiguous()
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=_F32)
        _K.maxpool_f32_bwd(dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), n, h, w, c, P, Q, k, s,
                           _st())
        return dx, None, None


def max_pool2d(x, kernel=2, stride=2, padding=0):
    _check(x)
    if padding not in (0, "valid", "VALID") or stride < kernel:
        raise ValueError("fp32 native max_pool2d: VALID, non-overlapping windows only")
    return _MaxPoolF32.apply(x, int(kernel), int(stride))


class _ClippedXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, onehot):
        z = logits.detach().to(_F32).contiguous()
        t = onehot.detach().to(_F32).contiguous()
        B, V = z.shape
        rows = torch.empty(B, device=z.device, dtype=_F32)
        dz = torch.empty_like(z)
        _K.clipped_xent(z.data_ptr(), t.data_ptr(), B, V, rows.data_ptr(), dz.data_ptr(), 1.0,
                        _st())
        ctx.save_for_backward(dz)
        ctx.dt = logits.dtype
        return rows.sum()

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        return (dz * g).to(ctx.dt), None


def softmax_cross_entropy_clipped_sum(logits, onehot):
    """templates/00_mnist_replica.py:160-164: -sum(t * log(clip(softmax(z), 1e-10, 1)))."""
    return _ClippedXent.apply(logits, onehot)
