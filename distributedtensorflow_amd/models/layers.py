"""tf.layers-compatible layer objects (names -> checkpoint keys) on top of :mod:`..ops`.

The reference builds its CNN with ``tf.layers.conv2d / max_pooling2d / dense``
(``run_mnist_distributed.py:52-69``) whose variables are named ``conv2d/kernel``,
``conv2d/bias``, ``conv2d_1/kernel`` ... (auto-uniquified per graph).  :class:`NameScope`
reproduces that naming so checkpoints written here carry the same keys.

Internal storage layouts are chosen for the HIP kernels; ``to_tf``/``from_tf`` in
:mod:`..train.checkpoint` convert:
  * conv kernel: internal ``[K, R, S, C]``  <->  TF ``[R, S, C, K]`` (HWIO)
  * dense kernel: internal ``[out, in]``     <->  TF ``[in, out]``
"""
from __future__ import annotations

import contextlib
import math
import threading

import torch
import torch.nn as nn

from .. import ops

_tls = threading.local()


class NameScope:
    """Per-model counter producing tf.layers-style unique names (``dense``, ``dense_1``...)."""

    def __init__(self, prefix: str = ""):
        self.prefix = prefix
        self.counts: dict[str, int] = {}

    def unique(self, base: str) -> str:
        n = self.counts.get(base, 0)
        self.counts[base] = n + 1
        name = base if n == 0 else f"{base}_{n}"
        return f"{self.prefix}/{name}" if self.prefix else name


@contextlib.contextmanager
def name_scope(prefix: str = ""):
    prev = getattr(_tls, "scope", None)
    _tls.scope = NameScope(prefix)
    try:
        yield _tls.scope
    finally:
        _tls.scope = prev


def _unique(base: str, name: str | None) -> str:
    if name is not None:
        return name
    scope = getattr(_tls, "scope", None)
    if scope is None:
        _tls.scope = scope = NameScope()
    return scope.unique(base)


def _tag(p, name, layout=None):
    p._dtf_name = name
    p._dtf_layout = layout
    return p


def glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int, gen=None):
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        t.uniform_(-limit, limit, generator=gen)
    return t


def truncated_normal_(t: torch.Tensor, stddev: float, gen=None):
    """TF truncated_normal: N(0, stddev) re-drawn outside +-2 stddev (vectorised inverse-CDF
    sampling; O(numel), no rejection loop)."""
    with torch.no_grad():
        if gen is None:
            torch.nn.init.trunc_normal_(t, 0.0, stddev, -2 * stddev, 2 * stddev)
        else:
            lo, hi = 0.5 * (1 + math.erf(-2 / math.sqrt(2))), 0.5 * (1 + math.erf(2 / math.sqrt(2)))
            u = torch.empty_like(t).uniform_(lo, hi, generator=gen)
            t.copy_(torch.erfinv(2 * u - 1) * math.sqrt(2) * stddev)
            t.clamp_(-2 * stddev, 2 * stddev)
    return t


def he_normal_(t, fan_in, gen=None):
    with torch.no_grad():
        t.normal_(0.0, math.sqrt(2.0 / fan_in), generator=gen)
    return t


class Layer(nn.Module):
    def variables_tf(self):
        """Yield (tf_name, tensor, layout) for params and non-trainable state."""
        for p in list(self.parameters(recurse=False)) + list(self.buffers(recurse=False)):
            if hasattr(p, "_dtf_name"):
                yield p._dtf_name, p, p._dtf_layout


class Conv2D(Layer):
    """tf.layers.conv2d: NHWC, kernel [K,R,S,C] internally, optional bias + ReLU."""

    def __init__(self, in_channels, filters, kernel_size, strides=1, padding="same",
                 activation=None, use_bias=True, name=None, init="glorot"):
        super().__init__()
        kh, kw = (kernel_size, kernel_size) if isinstance(kernel_size, int) else kernel_size
        self.name = _unique("conv2d", name)
        self.strides = strides
        self.padding = padding
        self.relu = activation in ("relu", torch.relu)
        self.kernel = _tag(nn.Parameter(torch.empty(filters, kh, kw, in_channels)),
                           f"{self.name}/kernel", "KRSC")
        fan_in = kh * kw * in_channels
        if init == "he":
            he_normal_(self.kernel.data, fan_in)
        else:
            glorot_uniform_(self.kernel.data, fan_in, kh * kw * filters)
        if use_bias:
            self.bias = _tag(nn.Parameter(torch.zeros(filters)), f"{self.name}/bias")
        else:
            self.bias = None

    def forward(self, x):
        if self.bias is not None or self.relu:
            # bias + ReLU fused into the conv epilogue on the native path
            return ops.conv2d_bias_relu(x, self.kernel, self.bias, self.strides, self.padding,
                                        self.relu)
        return ops.conv2d(x, self.kernel, self.strides, self.padding)


class Dense(Layer):
    """tf.layers.dense: y = x @ W + b, kernel stored [out, in] internally."""

    def __init__(self, in_units, units, activation=None, use_bias=True, name=None,
                 kernel_init=None, kernel_stddev=None):
        super().__init__()
        self.name = _unique("dense", name)
        self.relu = activation in ("relu", torch.relu)
        self.kernel = _tag(nn.Parameter(torch.empty(units, in_units)), f"{self.name}/kernel", "OI")
        if kernel_stddev is not None:
            truncated_normal_(self.kernel.data, kernel_stddev)
        else:
            glorot_uniform_(self.kernel.data, in_units, units)
        self.bias = _tag(nn.Parameter(torch.zeros(units)), f"{self.name}/bias") if use_bias else None

    def forward(self, x):
        return ops.dense(x, self.kernel, self.bias, self.relu)


class BatchNormalization(Layer):
    """tf.layers.batch_normalization over the channel axis with fused (+add) (+ReLU)."""

    def __init__(self, channels, momentum=0.997, epsilon=1e-5, name=None, gamma_init=1.0):
        super().__init__()
        self.name = _unique("batch_normalization", name)
        self.momentum = momentum
        self.epsilon = epsilon
        self.gamma = _tag(nn.Parameter(torch.full((channels,), float(gamma_init))),
                          f"{self.name}/gamma")
        self.beta = _tag(nn.Parameter(torch.zeros(channels)), f"{self.name}/beta")
        self.register_buffer("moving_mean", torch.zeros(channels))
        self.register_buffer("moving_variance", torch.ones(channels))
        _tag(self.moving_mean, f"{self.name}/moving_mean")
        _tag(self.moving_variance, f"{self.name}/moving_variance")

    def _apply(self, fn, *a, **k):  # keep tags across .to()/.cuda()
        out = super()._apply(fn, *a, **k)
        _tag(self.moving_mean, f"{self.name}/moving_mean")
        _tag(self.moving_variance, f"{self.name}/moving_variance")
        return out

    def forward(self, x, relu=False, residual=None, residual_to_conv=False, defer=False):
        return ops.batch_norm(x, self.gamma, self.beta, self.moving_mean, self.moving_variance,
                              self.training, self.momentum, self.epsilon, relu, residual,
                              residual_to_conv, defer)


class MaxPooling2D(Layer):
    def __init__(self, pool_size=2, strides=2, padding="valid", name=None):
        super().__init__()
        self.name = _unique("max_pooling2d", name)
        self.pool_size, self.strides, self.padding = pool_size, strides, padding

    def forward(self, x):
        return ops.max_pool2d(x, self.pool_size, self.strides, self.padding)


def collect_variables(module: nn.Module):
    """Ordered list of (tf_name, tensor, layout) over a module tree (creation order)."""
    seen = set()
    out = []
    for m in module.modules():
        if isinstance(m, Layer):
            for name, t, layout in m.variables_tf():
                if id(t) in seen:
                    continue
                seen.add(id(t))
                out.append((name, t, layout))
    return out
