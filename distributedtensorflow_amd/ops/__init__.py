"""Op layer: NHWC / bf16 ops backed by hand-written HIP (gfx950) kernels.

Dispatch rule (no multi-backend indirection on the GPU):
  * CUDA (HIP) tensors  -> :mod:`.native` (our HIP kernels).  If the compiled extension is
    missing this RAISES; it never silently falls back to PyTorch.
  * CPU tensors         -> :mod:`.reference` (PyTorch CPU), the OneDevice("/cpu:0") path.
  * ``set_backend("reference")`` forces the PyTorch path everywhere.  It exists for the
    stock-PyTorch comparator in ``bench.py --impl torch`` and for numerics tests.
"""
from __future__ import annotations

import os

import torch

from . import reference

_BACKEND = os.environ.get("DTF_OPS_BACKEND", "auto")   # auto | native | reference


def set_backend(name: str):
    global _BACKEND
    if name not in ("auto", "native", "reference"):
        raise ValueError(name)
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


def _use_native(t: torch.Tensor) -> bool:
    if _BACKEND == "reference":
        return False
    if _BACKEND == "native":
        return True
    return t.is_cuda


def _native():
    from . import native
    return native


def end_step():
    """Release the native ops' deferred-work records of the step whose backward just returned
    (:mod:`.records`: no record outlives its step); called by ``Optimizer.compute_gradients``.
    Returns the number released (0 when no native op ran)."""
    import sys
    m = sys.modules.get(__name__ + ".records")
    return m.end_step() if m is not None else 0


def _f32(t: torch.Tensor) -> bool:
    """fp32 GPU tensors run the fp32 HIP kernels (csrc/kernels/f32.hip): the reference
    workload at the reference's precision."""
    return _use_native(t) and t.dtype == torch.float32


def _native_f32():
    from . import native_f32
    return native_f32


class GradShare:
    """Marks the convs that read ONE input tensor (a projection block's x feeds both the 1x1
    shortcut conv and c1): on the native path their data gradients accumulate into one buffer
    in the dgrad epilogue instead of being summed by autograd with a separate add kernel.
    Create one per forward call; ``n`` = number of convs sharing the input."""

    def __init__(self, n: int):
        self.n = n
        self.left = n
        self.buf = None


def conv2d(x, w, stride=1, padding=0, bn_stats=False, grad_share=None):
    """``bn_stats``: a training-mode batch_norm consumes the result (native path fuses the BN
    statistics into the conv epilogue; ignored by the reference path).  ``grad_share``: a
    :class:`GradShare` common to every conv reading ``x`` (native path only)."""
    if _f32(x):
        return _native_f32().conv2d(x, w, stride, padding)
    if _use_native(x):
        return _native().conv2d(x, w, stride, padding, bn_stats, grad_share)
    return reference.conv2d(x, w, stride, padding)


def conv2d_bias_relu(x, w, bias=None, stride=1, padding=0, relu=True):
    """relu(conv2d(x, w) + bias): tf.layers.conv2d with ``activation=tf.nn.relu``.  Native path:
    bias and ReLU in the conv kernel's epilogue; backward ReluGrad + BiasAddGrad fused."""
    if _f32(x):
        return _native_f32().conv2d_bias_relu(x, w, bias, stride, padding, relu)
    if _use_native(x):
        return _native().conv2d_bias_relu(x, w, bias, stride, padding, relu)
    y = reference.conv2d(x, w, stride, padding)
    if bias is not None:
        y = y + bias.to(y.dtype)
    return reference.relu(y) if relu else y


def batch_norm(x, gamma, beta, running_mean=None, running_var=None, training=True,
               momentum=0.997, eps=1e-5, relu=False, residual=None, residual_to_conv=False,
               defer=False):
    """``residual_to_conv``: the residual tensor is also the input of a stride-1 conv whose
    data-gradient kernel will add d(residual) in its epilogue (native path; identity shortcuts).
    ``defer``: the result's only consumer is a 3x3 conv, which may apply this BN + ReLU on its
    input load instead of a separate apply pass (native path)."""
    if _use_native(x):
        return _native().batch_norm(x, gamma, beta, running_mean, running_var, training,
                                    momentum, eps, relu, residual, residual_to_conv, defer)
    return reference.batch_norm(x, gamma, beta, running_mean, running_var, training,
                                momentum, eps, relu, residual)


def batch_norm_relu_conv1x1(x, gamma, beta, running_mean, running_var, w, momentum=0.997,
                            eps=1e-5, lazy_out=False):
    """conv2d(relu(batch_norm(x, training=True)), w) for a 1x1 stride-1 conv.  Native path (when
    the conv runs on the row-streaming GEMM): one fused op, the BN output is written once by the
    GEMM instead of by a separate apply pass.  Else the two ops.  ``lazy_out``: the caller's
    only consumer of the result is a residual BatchNorm + ReLU (a bottleneck's c3), which may
    recompute the conv output instead of reading it (native: never stored)."""
    if _use_native(x) and _native().bn_relu_conv1x1_ok(x, w):
        return _native().bn_relu_conv1x1(x, gamma, beta, running_mean, running_var, w, momentum,
                                         eps, lazy_out)
    y = batch_norm(x, gamma, beta, running_mean, running_var, True, momentum, eps, relu=True)
    return conv2d(y, w, 1, 0, bn_stats=True)


def batch_norm_add_batch_norm(x, gamma, beta, running_mean, running_var, xp, gamma_p, beta_p,
                              running_mean_p, running_var_p, training=True, momentum=0.997,
                              eps=1e-5):
    """relu(batch_norm(x) + batch_norm(xp)): a ResNet projection block's output.  Native path:
    one fused op (the shortcut BN's output is never stored; one backward pass for both BNs)."""
    if _use_native(x):
        return _native().batch_norm_add_batch_norm(x, gamma, beta, running_mean, running_var, xp,
                                                   gamma_p, beta_p, running_mean_p,
                                                   running_var_p, training, momentum, eps)
    sc = reference.batch_norm(xp, gamma_p, beta_p, running_mean_p, running_var_p, training,
                              momentum, eps, False, None)
    return reference.batch_norm(x, gamma, beta, running_mean, running_var, training, momentum,
                                eps, True, sc)


def batch_norm_relu_max_pool(x, gamma, beta, running_mean=None, running_var=None, training=True,
                             momentum=0.997, eps=1e-5, kernel=3, stride=2, padding=1):
    """max_pool2d(batch_norm(x, relu=True)): the ResNet stem's BN -> ReLU -> 3x3/2 max-pool.
    Native path: one fused kernel that never stores the BN output."""
    if _use_native(x):
        return _native().batch_norm_relu_max_pool(x, gamma, beta, running_mean, running_var,
                                                  training, momentum, eps, kernel, stride, padding)
    y = reference.batch_norm(x, gamma, beta, running_mean, running_var, training, momentum, eps,
                             True, None)
    return max_pool2d(y, kernel, stride, padding)


def relu(x):
    if _use_native(x):
        return _native().relu(x)
    return reference.relu(x)


def max_pool2d(x, kernel=2, stride=2, padding=0):
    if _f32(x):
        return _native_f32().max_pool2d(x, kernel, stride, padding)
    if _use_native(x):
        return _native().max_pool2d(x, kernel, stride, padding)
    return reference.max_pool2d(x, kernel, stride, padding)


def global_avg_pool(x):
    if _use_native(x):
        return _native().global_avg_pool(x)
    return reference.global_avg_pool(x)


def dense(x, w, b=None, relu=False, impl=None, layout="OI"):
    """``impl`` (native path): None/"native" = the hand-written MFMA GEMM with fused bias/ReLU
    epilogues (tf.layers.dense); "library" = the bias-in-epilogue form BERT uses: its forward and
    data gradient run on our persistent MFMA GEMM (gemm_pp2) for every shape that kernel takes
    (N % 8 == 0, K % 64 == 0 -- all BERT-base layers, the tied decoder on its padded vocabulary
    included) and fall back to hipBLASLt only for other shapes.
    ``layout``: "OI" (kernel [out, in], tf.layers / BERT) or "IO" ([in, out], the MLP template's
    ``tf.nn.xw_plus_b`` weights)."""
    if _f32(x):
        return _native_f32().dense(x, w, b, relu, layout)
    if layout == "IO":
        w = w.t()
        if _use_native(x):
            w = w.contiguous()
    if _use_native(x):
        return _native().dense(x, w, b, relu, impl)
    return reference.dense(x, w, b, relu)


def sparse_softmax_cross_entropy(logits, labels):
    if _use_native(logits):
        return _native().sparse_softmax_cross_entropy(logits, labels)
    return reference.sparse_softmax_cross_entropy(logits, labels)


def softmax_cross_entropy_clipped_sum(logits, onehot):
    """The MLP template's loss (templates/00_mnist_replica.py:160-164), a batch SUM."""
    if _use_native(logits):
        return _native_f32().softmax_cross_entropy_clipped_sum(logits, onehot)
    return reference.softmax_cross_entropy_clipped_sum(logits, onehot)


def layer_norm(x, gamma, beta, eps=1e-12):
    if _use_native(x):
        return _native().layer_norm(x, gamma, beta, eps)
    return reference.layer_norm(x, gamma, beta, eps)


def gelu(x):
    if _use_native(x):
        return _native().gelu(x)
    return reference.gelu(x)


def attention(q, k, v, mask=None, scale=None):
    if _use_native(q):
        return _native().attention(q, k, v, mask, scale)
    return reference.attention(q, k, v, mask, scale)


def dropout(x, p, training=True):
    return reference.dropout(x, p, training)


def _nlp():
    from . import native_nlp
    return native_nlp


def bias_dropout_add_layer_norm(a, bias, residual, gamma, beta, p=0.0, training=True, eps=1e-12,
                                residual_to_dense=False):
    """LN(dropout(a + bias) + residual): the BERT sub-layer output, one fused kernel.
    ``residual_to_dense``: the caller guarantees ``residual`` is also the input of a later
    :func:`dense` (native path: that GEMM's dgrad then accumulates d(residual) with beta = 1
    instead of autograd adding the two bf16 gradients)."""
    if _use_native(a):
        return _nlp().bias_dropout_add_layer_norm(a, bias, residual, gamma, beta, p, training, eps,
                                                  residual_to_dense)
    return reference.bias_dropout_add_layer_norm(a, bias, residual, gamma, beta, p, training, eps)


def embedding_layer_norm(ids, token_type_ids, word, pos, typ, gamma, beta, p=0.0, training=True,
                         eps=1e-12, dtype=None):
    """dropout(LN(word[ids] + pos + type[tt])) -> [B*S, H]."""
    if _use_native(word):
        return _nlp().embedding_layer_norm(ids, token_type_ids, word, pos, typ, gamma, beta, p,
                                           training, eps)
    return reference.embedding_layer_norm(ids, token_type_ids, word, pos, typ, gamma, beta, p,
                                          training, eps, dtype=dtype)


def bias_gelu(a, bias=None):
    if _use_native(a):
        return _nlp().bias_gelu(a, bias)
    return reference.bias_gelu(a, bias)


def bias_gelu_dense(a, bias, w):
    """gelu(a + bias) @ w^T (w [out, in]): BERT's FFN after its first GEMM.  Native: the data
    gradient of a is one GEMM pass with the GELU derivative and the bias-gradient column sums in
    its epilogue."""
    if _use_native(a):
        return _native().bias_gelu_dense(a, bias, w)
    return reference.dense(reference.bias_gelu(a, bias), w)


def dense_gelu_dense(x, w1, b1, w2):
    """gelu(x @ w1^T + b1) @ w2^T (w [out, in]): BERT's FFN.  Native: the first GEMM carries
    the bias + GELU in its epilogue and also writes the pre-activation for the backward."""
    if _use_native(x):
        return _native().dense_gelu_dense(x, w1, b1, w2)
    return reference.dense(reference.bias_gelu(reference.dense(x, w1), b1), w2)


def attention_qkv(qkv, mask, batch, seq_len, heads, p=0.0, training=True, scale=None):
    """Multi-head self-attention straight from the fused QKV projection output."""
    if _use_native(qkv):
        return _nlp().attention_qkv(qkv, mask, batch, seq_len, heads, p, training, scale)
    return reference.attention_qkv(qkv, mask, batch, seq_len, heads, p, training, scale)


def mlm_loss(logits, labels, weights=None, vocab=None):
    """Weighted masked-LM cross-entropy.  ``vocab``: the class count when the logits rows are
    padded past it (BERT's tied decoder runs on a vocabulary padded to a multiple of 64)."""
    if _use_native(logits):
        return _nlp().mlm_loss(logits, labels, weights, vocab)
    return reference.mlm_loss(logits, labels, weights, vocab)


# ----------------------------------------------------------------------------- variable fence
# A colocated parameter server gathers the updated variable shards AFTER the optimizer step,
# asynchronously, bucket by bucket, while the next forward already runs (parallel/ps_strategy.py).
# Every op that reads variables first passes them to the fence, which makes the compute stream
# wait for exactly the gather that writes them (nothing to do -- and no scan -- when no gather
# is pending: the fence is then None).
_PARAM_FENCE = None


def set_param_fence(fn):
    global _PARAM_FENCE
    _PARAM_FENCE = fn


_TRACER = None      # train/saved_model.py: records ops applied to symbolic graph tensors


def set_tracer(tracer):
    global _TRACER
    _TRACER = tracer


def _dispatch(name, fn, fenced):
    import functools

    @functools.wraps(fn)
    def op(*args, **kw):
        if _TRACER is not None and args and isinstance(args[0], _TRACER.Tensor):
            return _TRACER.call(name, args, kw)
        if fenced and _PARAM_FENCE is not None:
            _PARAM_FENCE(args, kw)
        return fn(*args, **kw)
    return op


# EVERY public op entry point passes through the fence: a per-op allow-list went stale once
# already (bias_gelu_dense read an un-gathered W2 shadow), and the fence costs one
# global load when no gather is pending and an attribute scan of the arguments otherwise.
_OPS = ("conv2d", "conv2d_bias_relu", "batch_norm", "batch_norm_add_batch_norm",
        "batch_norm_relu_conv1x1", "batch_norm_relu_max_pool", "dense", "layer_norm",
        "bias_dropout_add_layer_norm", "embedding_layer_norm", "bias_gelu", "bias_gelu_dense",
        "dense_gelu_dense", "relu", "max_pool2d", "global_avg_pool", "sparse_softmax_cross_entropy",
        "softmax_cross_entropy_clipped_sum", "gelu", "attention", "dropout", "attention_qkv",
        "mlm_loss")
_FENCED = _OPS
for _name in _OPS:
    globals()[_name] = _dispatch(_name, globals()[_name], True)
del _name

__all__ = [
    "set_backend", "get_backend", "GradShare", "conv2d", "conv2d_bias_relu", "batch_norm", "relu",
    "batch_norm_add_batch_norm", "batch_norm_relu_conv1x1",
    "max_pool2d", "global_avg_pool", "dense", "sparse_softmax_cross_entropy",
    "softmax_cross_entropy_clipped_sum", "layer_norm", "gelu", "attention", "dropout",
    "bias_dropout_add_layer_norm", "embedding_layer_norm", "bias_gelu", "bias_gelu_dense",
    "dense_gelu_dense", "attention_qkv", "mlm_loss",
]
