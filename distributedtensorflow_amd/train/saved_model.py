"""TensorFlow SavedModel export with a real inference GraphDef (north star).

The reference checkpoints through ``MonitoredTrainingSession(checkpoint_dir=...)``
(``/root/reference/templates/00_between_graph_replication_async_mnist.py:45``); the north star
asks for TF's checkpoint / SavedModel layout.  A TF1-format SavedModel is

    export_dir/saved_model.pb                       SavedModel{MetaGraphDef}
    export_dir/variables/variables.index / .data-*  a checkpoint-V2 bundle (io/bundle.py)

and the MetaGraphDef written here carries what TF's loaders and TF Serving need:

* a ``GraphDef`` of the model's INFERENCE computation in stock TF ops -- ``Placeholder`` input,
  resource variables (``VarHandleOp`` + ``ReadVariableOp``, shared_name = the checkpoint key),
  ``Conv2D`` (SAME / VALID / EXPLICIT padding), ``BiasAdd``, ``Relu``, ``FusedBatchNormV3``
  (is_training = false, moving statistics), ``AddV2``, ``PadV2`` + ``MaxPool``, ``Mean``,
  ``Reshape``, ``MatMul``, ``Softmax`` -- obtained by TRACING the model's forward: the model is
  called on a symbolic tensor and every :mod:`..ops` call records its node;
* the saver subgraph (``save/Const`` filename, ``save/SaveV2`` + ``save/control_dependency``,
  ``save/RestoreV2`` -> ``AssignVariableOp`` per variable -> ``save/restore_all``) and the
  matching ``SaverDef`` (checkpoint format V2), so ``loader.load`` restores the variables;
* a ``serving_default`` ``SignatureDef`` (``tensorflow/serving/predict``): input ``images``,
  outputs ``logits`` and ``probabilities``.

TensorFlow itself is not importable here, so the tests decode the protobufs with an independent
wire-format reader and EXECUTE the graph with a small interpreter against the model's own
forward (tests/test_saved_model.py) -- TF parity of the loader itself is unpinned.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..io import pbwire as pb

DT_FLOAT, DT_INT32, DT_STRING, DT_RESOURCE = 1, 3, 7, 20
PREDICT = "tensorflow/serving/predict"


# ----------------------------------------------------------------------------- attr encoders

def _shape(dims):
    if dims is None:
        return pb.f_bool(3, True)                          # unknown_rank
    return b"".join(pb.f_msg(2, pb.f_int(1, -1 if d is None else int(d))) for d in dims)


def a_type(t):
    return pb.f_int(6, t)


def a_str(s):
    return pb.f_bytes(2, s.encode() if isinstance(s, str) else s)


def a_int(i):
    return pb.f_int(3, i)


def a_float(f):
    return pb.f_float(4, f)


def a_bool(b):
    return pb.f_bool(5, b)


def a_shape(dims):
    return pb.f_msg(7, _shape(dims))


def a_ints(vals):
    return pb.f_msg(1, pb.f_packed_ints(3, vals))


def a_types(vals):
    return pb.f_msg(1, pb.f_packed_ints(6, vals))


def a_tensor(arr):
    """TensorProto of a numpy array (float32 / int32 content, or a string list)."""
    arr = np.asarray(arr)
    if arr.dtype.kind in ("U", "S", "O"):
        body = pb.f_int(1, DT_STRING) + pb.f_msg(2, _shape(arr.shape)) + \
            b"".join(pb.f_bytes(8, str(s).encode()) for s in arr.reshape(-1))
    else:
        dt = DT_INT32 if arr.dtype.kind in "iu" else DT_FLOAT
        arr = arr.astype(np.int32 if dt == DT_INT32 else np.float32)
        body = pb.f_int(1, dt) + pb.f_msg(2, _shape(arr.shape)) + \
            pb.f_bytes(4, arr.astype("<" + arr.dtype.str[1:]).tobytes())
    return pb.f_msg(8, body)


# ----------------------------------------------------------------------------- graph builder

class GraphDef:
    def __init__(self):
        self.nodes = []
        self.names = set()

    def unique(self, base):
        name, k = base, 0
        while name in self.names:
            k += 1
            name = f"{base}_{k}"
        return name

    def add(self, op, name, inputs=(), **attrs):
        name = self.unique(name)
        self.names.add(name)
        self.nodes.append((name, op, list(inputs), attrs))
        return name

    def const(self, name, arr):
        arr = np.asarray(arr)
        dt = DT_STRING if arr.dtype.kind in ("U", "S", "O") else \
            (DT_INT32 if arr.dtype.kind in "iu" else DT_FLOAT)
        return self.add("Const", name, dtype=a_type(dt), value=a_tensor(arr))

    def encode(self, producer=134):
        out = b""
        for name, op, inputs, attrs in self.nodes:
            body = pb.f_str(1, name) + pb.f_str(2, op) + b"".join(pb.f_str(3, i) for i in inputs)
            body += pb.f_map(5, attrs, lambda f, v: pb.f_msg(f, v))
            out += pb.f_msg(1, body)
        return out + pb.f_msg(4, pb.f_int(1, producer) + pb.f_int(2, 12))


# ----------------------------------------------------------------------------- tracer

class _Sym:
    """A symbolic NHWC graph tensor flowing through the model's forward."""

    def __init__(self, tracer, name, shape):
        self._t, self.name, self._shape = tracer, name, tuple(shape)
        self.is_cuda = False
        self.requires_grad = False
        self.dtype = torch.float32

    @property
    def shape(self):
        return self._shape

    def dim(self):
        return len(self._shape)

    def float(self):
        return self

    def to(self, *a, **k):
        return self

    def contiguous(self):
        return self

    def reshape(self, *shape):
        if len(shape) == 1 and isinstance(shape, (tuple, list)) and \
                isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        shape = tuple(-1 if s is None else int(s) for s in shape)
        g = self._t.g
        c = g.const(self.name.split(":")[0] + "/shape", np.array(shape, dtype=np.int32))
        n = g.add("Reshape", "Reshape", [self.name, c], T=a_type(DT_FLOAT),
                  Tshape=a_type(DT_INT32))
        known = [s for s in shape if s != -1]
        total = int(np.prod([s for s in self._shape if s is not None and s > 0]))
        out = tuple(None if s == -1 else s for s in shape)
        if -1 in shape and None not in self._shape and known:
            out = tuple(total // int(np.prod(known)) if s == -1 else s for s in shape)
        return _Sym(self._t, n + ":0", out)

    view = reshape


class Tracer:
    Tensor = _Sym

    def __init__(self, model):
        from ..models.layers import collect_variables
        self.g = GraphDef()
        self.vars = {}          # id(tensor) -> (tf_name, np value in TF layout)
        self.var_nodes = {}
        from .checkpoint import to_tf_layout
        for name, t, layout in collect_variables(model):
            val = to_tf_layout(t.detach().float().cpu(), layout).contiguous().numpy()
            self.vars[id(t)] = (name, val)

    # variables: VarHandleOp + ReadVariableOp, created on first use
    def read(self, t):
        if t is None:
            return None
        name, val = self.vars[id(t)]
        if name not in self.var_nodes:
            h = self.g.add("VarHandleOp", name, container=a_str(""), shared_name=a_str(name),
                           dtype=a_type(DT_FLOAT), shape=a_shape(val.shape))
            r = self.g.add("ReadVariableOp", f"{name}/Read/ReadVariableOp", [h],
                           dtype=a_type(DT_FLOAT))
            self.var_nodes[name] = (h, r + ":0", val)
        return self.var_nodes[name][1]

    def _nhwc(self, x, name, c):
        return _Sym(self, name + ":0", tuple(x.shape[:-1]) + (c,))

    # -- op emitters (signatures mirror ops/__init__.py)
    def call(self, name, args, kw):
        fn = getattr(self, "op_" + name, None)
        if fn is None:
            raise NotImplementedError(f"SavedModel export: op {name!r} has no graph emitter")
        return fn(*args, **kw)

    def _conv(self, x, w, stride, padding):
        s = stride if isinstance(stride, int) else stride[0]
        k = self.vars[id(w)][1].shape            # HWIO
        attrs = {"T": a_type(DT_FLOAT), "strides": a_ints([1, s, s, 1]),
                 "data_format": a_str("NHWC"), "dilations": a_ints([1, 1, 1, 1]),
                 "use_cudnn_on_gpu": a_bool(True)}
        if isinstance(padding, str):
            attrs["padding"] = a_str(padding.upper())
            ph = pw = (k[0] - 1) // 2 if padding.lower() == "same" else 0
            same = padding.lower() == "same"
        else:
            p = padding if isinstance(padding, int) else padding[0]
            attrs["padding"] = a_str("EXPLICIT")
            attrs["explicit_paddings"] = a_ints([0, 0, p, p, p, p, 0, 0])
            ph = pw = p
            same = False
        n = self.g.add("Conv2D", "Conv2D", [x.name, self.read(w)], **attrs)
        H, W = x.shape[1], x.shape[2]
        if same:
            Ho, Wo = -(-H // s), -(-W // s)
        else:
            Ho, Wo = (H + 2 * ph - k[0]) // s + 1, (W + 2 * pw - k[1]) // s + 1
        return _Sym(self, n + ":0", (x.shape[0], Ho, Wo, k[3]))

    def _bias_relu(self, y, bias, relu):
        if bias is not None:
            y = _Sym(self, self.g.add("BiasAdd", "BiasAdd", [y.name, self.read(bias)],
                                      T=a_type(DT_FLOAT), data_format=a_str("NHWC")) + ":0",
                     y.shape)
        if relu:
            y = self.op_relu(y)
        return y

    def op_relu(self, x):
        return _Sym(self, self.g.add("Relu", "Relu", [x.name], T=a_type(DT_FLOAT)) + ":0",
                    x.shape)

    def op_conv2d(self, x, w, stride=1, padding=0, bn_stats=False, grad_share=None):
        return self._conv(x, w, stride, padding)

    def op_conv2d_bias_relu(self, x, w, bias=None, stride=1, padding=0, relu=True):
        return self._bias_relu(self._conv(x, w, stride, padding), bias, relu)

    def _bn(self, x, gamma, beta, mean, var, eps):
        n = self.g.add("FusedBatchNormV3", "FusedBatchNormV3",
                       [x.name, self.read(gamma), self.read(beta), self.read(mean),
                        self.read(var)],
                       T=a_type(DT_FLOAT), U=a_type(DT_FLOAT), epsilon=a_float(eps),
                       data_format=a_str("NHWC"), is_training=a_bool(False))
        # (no exponential_avg_factor: that attr is TF >= 2.2, and a TF 1.15 loader -- the
        # MetaGraph's declared version -- rejects NodeDefs with attrs its op registry lacks)
        return _Sym(self, n + ":0", x.shape)

    def _add(self, a, b):
        return _Sym(self, self.g.add("AddV2", "add", [a.name, b.name], T=a_type(DT_FLOAT)) + ":0",
                    a.shape)

    def op_batch_norm(self, x, gamma, beta, running_mean=None, running_var=None, training=True,
                      momentum=0.997, eps=1e-5, relu=False, residual=None,
                      residual_to_conv=False, defer=False):
        y = self._bn(x, gamma, beta, running_mean, running_var, eps)
        if residual is not None:
            y = self._add(y, residual)
        return self.op_relu(y) if relu else y

    def op_batch_norm_add_batch_norm(self, x, gamma, beta, running_mean, running_var, xp,
                                     gamma_p, beta_p, running_mean_p, running_var_p,
                                     training=True, momentum=0.997, eps=1e-5):
        y = self._add(self._bn(x, gamma, beta, running_mean, running_var, eps),
                      self._bn(xp, gamma_p, beta_p, running_mean_p, running_var_p, eps))
        return self.op_relu(y)

    def op_batch_norm_relu_max_pool(self, x, gamma, beta, running_mean=None, running_var=None,
                                    training=True, momentum=0.997, eps=1e-5, kernel=3, stride=2,
                                    padding=1):
        y = self.op_batch_norm(x, gamma, beta, running_mean, running_var, False, momentum, eps,
                               True)
        return self.op_max_pool2d(y, kernel, stride, padding)

    def op_max_pool2d(self, x, kernel=2, stride=2, padding=0):
        if isinstance(padding, str):
            p = (kernel - 1) // 2 if padding.lower() == "same" else 0
        else:
            p = padding
        src = x.name
        H, W = x.shape[1], x.shape[2]
        if p:
            pads = self.g.const("MaxPool/paddings",
                                np.array([[0, 0], [p, p], [p, p], [0, 0]], dtype=np.int32))
            lowest = self.g.const("MaxPool/lowest", np.array(np.finfo(np.float32).min,
                                                             dtype=np.float32))
            src = self.g.add("PadV2", "PadV2", [src, pads, lowest], T=a_type(DT_FLOAT),
                             Tpaddings=a_type(DT_INT32)) + ":0"
            H, W = H + 2 * p, W + 2 * p
        n = self.g.add("MaxPool", "MaxPool", [src], T=a_type(DT_FLOAT),
                       ksize=a_ints([1, kernel, kernel, 1]), strides=a_ints([1, stride, stride, 1]),
                       padding=a_str("VALID"), data_format=a_str("NHWC"))
        return _Sym(self, n + ":0", (x.shape[0], (H - kernel) // stride + 1,
                                     (W - kernel) // stride + 1, x.shape[3]))

    def op_global_avg_pool(self, x):
        axes = self.g.const("Mean/reduction_indices", np.array([1, 2], dtype=np.int32))
        n = self.g.add("Mean", "Mean", [x.name, axes], T=a_type(DT_FLOAT),
                       Tidx=a_type(DT_INT32), keep_dims=a_bool(False))
        return _Sym(self, n + ":0", (x.shape[0], x.shape[3]))

    def op_dense(self, x, w, b=None, relu=False, impl=None, layout="OI"):
        k = self.vars[id(w)][1].shape              # TF layout [in, out]
        n = self.g.add("MatMul", "MatMul", [x.name, self.read(w)], T=a_type(DT_FLOAT),
                       transpose_a=a_bool(False), transpose_b=a_bool(False))
        return self._bias_relu(_Sym(self, n + ":0", (x.shape[0], k[1])), b, relu)


# ----------------------------------------------------------------------------- export

def _saver_nodes(g, names_vals, handles):
    """TF1 Saver subgraph over the resource variables (checkpoint format V2)."""
    names = [n for n, _ in names_vals]
    prefix = g.const("save/Const", np.array("model", dtype=object))
    tn = g.const("save/SaveV2/tensor_names", np.array(names, dtype=object))
    ss = g.const("save/SaveV2/shape_and_slices", np.array([""] * len(names), dtype=object))
    reads = [handles[n][1] for n in names]
    save = g.add("SaveV2", "save/SaveV2", [prefix, tn, ss] + reads,
                 dtypes=a_types([DT_FLOAT] * len(names)))
    g.add("Identity", "save/control_dependency", [prefix, "^" + save], T=a_type(DT_STRING),
          _class=pb.f_msg(1, pb.f_bytes(2, f"loc:@{prefix}".encode())))
    rtn = g.const("save/RestoreV2/tensor_names", np.array(names, dtype=object))
    rss = g.const("save/RestoreV2/shape_and_slices", np.array([""] * len(names), dtype=object))
    restore = g.add("RestoreV2", "save/RestoreV2", [prefix, rtn, rss],
                    dtypes=a_types([DT_FLOAT] * len(names)))
    assigns = []
    for i, n in enumerate(names):
        ident = g.add("Identity", f"save/Identity_{i}", [f"{restore}:{i}"], T=a_type(DT_FLOAT))
        assigns.append(g.add("AssignVariableOp", f"save/AssignVariableOp_{i}",
                             [handles[n][0], ident], dtype=a_type(DT_FLOAT)))
    g.add("NoOp", "save/restore_all", ["^" + a for a in assigns])
    return prefix + ":0", "save/control_dependency:0", "save/restore_all"


def _tensor_info(name, dtype, dims):
    return pb.f_str(1, name) + pb.f_int(2, dtype) + pb.f_msg(3, _shape(dims))


def export_saved_model(export_dir, model, input_shape, tags=("serve",), input_name="images"):
    """Write ``saved_model.pb`` (graph + saver + serving signature) and ``variables/``.

    ``input_shape``: the model input with ``None`` for the batch dimension, e.g.
    ``(None, 784)`` for the MNIST models, ``(None, 224, 224, 3)`` for ResNet-50 (NHWC)."""
    from .. import ops
    _write_variables(export_dir, model)

    tracer = Tracer(model)
    g = tracer.g
    inp = g.add("Placeholder", "input", dtype=a_type(DT_FLOAT), shape=a_shape(input_shape))
    was_training = model.training
    model.eval()
    ops.set_tracer(tracer)
    try:
        out = model(_Sym(tracer, inp + ":0", input_shape))
    finally:
        ops.set_tracer(None)
        model.train(was_training)
    logits = g.add("Identity", "logits", [out.name], T=a_type(DT_FLOAT))
    probs = g.add("Softmax", "probabilities", [logits], T=a_type(DT_FLOAT))
    # every checkpointed variable gets a handle, used in the forward or not (moving statistics
    # of an unused layer still round-trip through the saver)
    for t_id, (name, val) in tracer.vars.items():
        if name not in tracer.var_nodes:
            h = g.add("VarHandleOp", name, container=a_str(""), shared_name=a_str(name),
                      dtype=a_type(DT_FLOAT), shape=a_shape(val.shape))
            r = g.add("ReadVariableOp", f"{name}/Read/ReadVariableOp", [h], dtype=a_type(DT_FLOAT))
            tracer.var_nodes[name] = (h, r + ":0", val)
    out_dims = list(out.shape)
    _write_saved_model(export_dir, g, tracer.var_nodes, tags,
                       {input_name: (inp + ":0", DT_FLOAT, input_shape)},
                       {"logits": (logits + ":0", DT_FLOAT, out_dims),
                        "probabilities": (probs + ":0", DT_FLOAT, out_dims)})
    return export_dir


def _write_saved_model(export_dir, g, var_nodes, tags, inputs, outputs):
    """saved_model.pb: MetaGraphDef{meta_info, graph_def (+ saver subgraph), saver_def,
    signature_def{"serving_default": inputs -> outputs}}; ``inputs`` / ``outputs`` map a
    signature key to (tensor name, dtype, dims)."""
    names_vals = sorted((n, v) for n, (_, _, v) in var_nodes.items())
    fname, save_t, restore_op = _saver_nodes(g, names_vals, var_nodes)
    meta_info = pb.f_str(1, "dtf-v1") + b"".join(pb.f_str(4, t) for t in tags) + \
        pb.f_str(5, "1.15.0") + pb.f_str(6, "distributedtensorflow_amd")
    saver_def = pb.f_str(1, fname) + pb.f_str(2, save_t) + pb.f_str(3, restore_op) + \
        pb.f_int(4, 5) + pb.f_bool(5, False) + pb.f_float(6, 10000.0) + pb.f_int(7, 2)
    sig = pb.f_map(1, {k: _tensor_info(*v) for k, v in inputs.items()},
                   lambda f, v: pb.f_msg(f, v)) + \
        pb.f_map(2, {k: _tensor_info(*v) for k, v in outputs.items()},
                 lambda f, v: pb.f_msg(f, v)) + pb.f_str(3, PREDICT)
    meta = pb.f_msg(1, meta_info) + pb.f_msg(2, g.encode()) + pb.f_msg(3, saver_def) + \
        pb.f_map(5, {"serving_default": sig}, lambda f, v: pb.f_msg(f, v))
    with open(os.path.join(export_dir, "saved_model.pb"), "wb") as f:
        f.write(pb.f_int(1, 1) + pb.f_msg(2, meta))


def _write_variables(export_dir, model):
    from .checkpoint import Saver
    os.makedirs(os.path.join(export_dir, "variables"), exist_ok=True)
    Saver(model, write_meta_graph=False).save(
        save_path=os.path.join(export_dir, "variables", "variables"))
    state = os.path.join(export_dir, "variables", "checkpoint")
    if os.path.exists(state):
        os.remove(state)


# ----------------------------------------------------------------------------- BERT

class _BertGraph:
    """Inference graph of :class:`~..models.bert.BertForPreTraining` in the op vocabulary of
    google-research/bert's ``modeling.py`` (TF 1.15): GatherV2 embeddings, moments-style
    LayerNorm (Mean / SquaredDifference / Rsqrt), per-head attention as Reshape + Transpose +
    BatchMatMulV2 + Softmax with the additive -10000 key mask, tanh-GELU, and the MLM head
    whose decoder is the word-embedding table (MatMul transpose_b).  The fused training kernels
    (QKV in one GEMM, flash attention, bias+dropout+residual+LN) do not exist in TF: each is
    lowered here to the stock ops computing the same function in inference mode."""

    def __init__(self, model, seq_len):
        from .checkpoint import to_tf_layout
        self.model, self.cfg, self.S = model, model.cfg, int(seq_len)
        if self.S > self.cfg.max_position_embeddings:
            raise ValueError(f"seq_len {self.S} > max_position_embeddings")
        self.g = GraphDef()
        self.vals = {}
        for name, t, layout in model.variables_tf():
            self.vals[name] = to_tf_layout(t.detach().float().cpu(), layout).contiguous().numpy()
        self.var_nodes = {}

    # helpers
    def var(self, name):
        if name not in self.var_nodes:
            val = self.vals[name]
            h = self.g.add("VarHandleOp", name, container=a_str(""), shared_name=a_str(name),
                           dtype=a_type(DT_FLOAT), shape=a_shape(val.shape))
            r = self.g.add("ReadVariableOp", f"{name}/Read/ReadVariableOp", [h],
                           dtype=a_type(DT_FLOAT))
            self.var_nodes[name] = (h, r + ":0", val)
        return self.var_nodes[name][1]

    def op(self, op, name, inputs, **attrs):
        return self.g.add(op, name, inputs, **attrs) + ":0"

    def c(self, name, arr):
        return self.g.const(name, arr) + ":0"

    def f(self, op, name, *inputs, **attrs):
        return self.op(op, name, list(inputs), T=a_type(DT_FLOAT), **attrs)

    def reshape(self, x, shape, name="Reshape"):
        return self.op("Reshape", name, [x, self.c(name + "/shape", np.array(shape, np.int32))],
                       T=a_type(DT_FLOAT), Tshape=a_type(DT_INT32))

    def transpose(self, x, perm, name="transpose"):
        return self.op("Transpose", name, [x, self.c(name + "/perm", np.array(perm, np.int32))],
                       T=a_type(DT_FLOAT), Tperm=a_type(DT_INT32))

    def dense(self, x, scope, transpose_b=False, kernel=None, bias=None):
        k = kernel or self.var(f"{scope}/kernel")
        y = self.f("MatMul", f"{scope}/MatMul", x, k, transpose_a=a_bool(False),
                   transpose_b=a_bool(transpose_b))
        return self.f("BiasAdd", f"{scope}/BiasAdd", y, bias or self.var(f"{scope}/bias"),
                      data_format=a_str("NHWC"))

    def layer_norm(self, x, scope, eps):
        axes = self.c(f"{scope}/moments/axes", np.array([-1], np.int32))
        mean = self.op("Mean", f"{scope}/moments/mean", [x, axes], T=a_type(DT_FLOAT),
                       Tidx=a_type(DT_INT32), keep_dims=a_bool(True))
        sq = self.f("SquaredDifference", f"{scope}/moments/SquaredDifference", x, mean)
        var = self.op("Mean", f"{scope}/moments/variance", [sq, axes], T=a_type(DT_FLOAT),
                      Tidx=a_type(DT_INT32), keep_dims=a_bool(True))
        ve = self.f("AddV2", f"{scope}/batchnorm/add", var,
                    self.c(f"{scope}/batchnorm/add/y", np.array(eps, np.float32)))
        rs = self.f("Rsqrt", f"{scope}/batchnorm/Rsqrt", ve)
        sc = self.f("Mul", f"{scope}/batchnorm/mul", rs, self.var(f"{scope}/gamma"))
        xs = self.f("Mul", f"{scope}/batchnorm/mul_1", x, sc)
        ms = self.f("Mul", f"{scope}/batchnorm/mul_2", mean, sc)
        sh = self.f("Sub", f"{scope}/batchnorm/sub", self.var(f"{scope}/beta"), ms)
        return self.f("AddV2", f"{scope}/batchnorm/add_1", xs, sh)

    def gelu(self, x, scope):
        """0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))) -- modeling.py's gelu."""
        x3 = self.f("Pow", f"{scope}/Pow", x, self.c(f"{scope}/Pow/y", np.array(3.0, np.float32)))
        t = self.f("Mul", f"{scope}/mul", x3, self.c(f"{scope}/mul/x",
                                                     np.array(0.044715, np.float32)))
        t = self.f("AddV2", f"{scope}/add", x, t)
        t = self.f("Mul", f"{scope}/mul_1", t, self.c(f"{scope}/mul_1/x",
                                                      np.array(np.sqrt(2 / np.pi), np.float32)))
        t = self.f("Tanh", f"{scope}/Tanh", t)
        t = self.f("AddV2", f"{scope}/add_1", t, self.c(f"{scope}/add_1/x",
                                                        np.array(1.0, np.float32)))
        t = self.f("Mul", f"{scope}/mul_2", t, self.c(f"{scope}/mul_2/x",
                                                      np.array(0.5, np.float32)))
        return self.f("Mul", f"{scope}/mul_3", x, t)

    def build(self):
        cfg, S, H = self.cfg, self.S, self.cfg.hidden_size
        nh, D = cfg.num_attention_heads, cfg.hidden_size // cfg.num_attention_heads
        eps = cfg.layer_norm_eps
        i32 = dict(dtype=a_type(DT_INT32), shape=a_shape([None, S]))
        ids = self.g.add("Placeholder", "input_ids", **i32) + ":0"
        tts = self.g.add("Placeholder", "token_type_ids", **i32) + ":0"
        msk = self.g.add("Placeholder", "input_mask", **i32) + ":0"
        self.inputs = {"input_ids": ids, "token_type_ids": tts, "input_mask": msk}
        ax0 = self.c("bert/embeddings/axis", np.array(0, np.int32))
        gather = dict(Tparams=a_type(DT_FLOAT), Tindices=a_type(DT_INT32),
                      Taxis=a_type(DT_INT32))
        word = self.var("bert/embeddings/word_embeddings")
        e = self.op("GatherV2", "bert/embeddings/GatherV2", [word, ids, ax0], **gather)
        t = self.op("GatherV2", "bert/embeddings/GatherV2_1",
                    [self.var("bert/embeddings/token_type_embeddings"), tts, ax0], **gather)
        pos = self.op("Slice", "bert/embeddings/Slice",
                      [self.var("bert/embeddings/position_embeddings"),
                       self.c("bert/embeddings/Slice/begin", np.array([0, 0], np.int32)),
                       self.c("bert/embeddings/Slice/size", np.array([S, -1], np.int32))],
                      T=a_type(DT_FLOAT), Index=a_type(DT_INT32))
        e = self.f("AddV2", "bert/embeddings/add", e, t)
        e = self.f("AddV2", "bert/embeddings/add_1", e, pos)
        x = self.layer_norm(e, "bert/embeddings/LayerNorm", eps)
        x = self.reshape(x, [-1, H], "bert/encoder/Reshape")
        m = self.op("Cast", "bert/encoder/Cast", [msk], SrcT=a_type(DT_INT32),
                    DstT=a_type(DT_FLOAT), Truncate=a_bool(False))
        m = self.f("Sub", "bert/encoder/sub", self.c("bert/encoder/sub/x",
                                                      np.array(1.0, np.float32)), m)
        m = self.f("Mul", "bert/encoder/mul", m, self.c("bert/encoder/mul/y",
                                                        np.array(-10000.0, np.float32)))
        m = self.reshape(m, [-1, 1, 1, S], "bert/encoder/mask")
        for li in range(cfg.num_hidden_layers):
            pre = f"bert/encoder/layer_{li}"
            heads = []
            for nm in ("query", "key", "value"):
                y = self.dense(x, f"{pre}/attention/self/{nm}")
                y = self.reshape(y, [-1, S, nh, D], f"{pre}/attention/self/{nm}/Reshape")
                heads.append(self.transpose(y, [0, 2, 1, 3], f"{pre}/attention/self/{nm}/T"))
            q, k, v = heads
            s = self.f("BatchMatMulV2", f"{pre}/attention/self/MatMul", q, k,
                       adj_x=a_bool(False), adj_y=a_bool(True))
            s = self.f("Mul", f"{pre}/attention/self/Mul", s,
                       self.c(f"{pre}/attention/self/Mul/y",
                              np.array(1.0 / np.sqrt(D), np.float32)))
            s = self.f("AddV2", f"{pre}/attention/self/add", s, m)
            p = self.f("Softmax", f"{pre}/attention/self/Softmax", s)
            ctx = self.f("BatchMatMulV2", f"{pre}/attention/self/MatMul_1", p, v,
                         adj_x=a_bool(False), adj_y=a_bool(False))
            ctx = self.transpose(ctx, [0, 2, 1, 3], f"{pre}/attention/self/transpose_3")
            ctx = self.reshape(ctx, [-1, H], f"{pre}/attention/self/Reshape_3")
            a = self.dense(ctx, f"{pre}/attention/output/dense")
            a = self.f("AddV2", f"{pre}/attention/output/add", a, x)
            x = self.layer_norm(a, f"{pre}/attention/output/LayerNorm", eps)
            h = self.gelu(self.dense(x, f"{pre}/intermediate/dense"), f"{pre}/intermediate/gelu")
            o = self.dense(h, f"{pre}/output/dense")
            o = self.f("AddV2", f"{pre}/output/add", o, x)
            x = self.layer_norm(o, f"{pre}/output/LayerNorm", eps)
        seq = self.reshape(x, [-1, S, H], "sequence_output")
        tr = self.gelu(self.dense(x, "cls/predictions/transform/dense"),
                       "cls/predictions/transform/gelu")
        tr = self.layer_norm(tr, "cls/predictions/transform/LayerNorm", eps)
        logits = self.dense(tr, "cls/predictions", transpose_b=True, kernel=word,
                            bias=self.var("cls/predictions/output_bias"))
        logits = self.reshape(logits, [-1, S, cfg.vocab_size], "mlm_logits")
        probs = self.f("Softmax", "mlm_probabilities", logits)
        self.outputs = {"sequence_output": (seq, [None, S, H]),
                        "mlm_logits": (logits, [None, S, cfg.vocab_size]),
                        "mlm_probabilities": (probs, [None, S, cfg.vocab_size])}
        # every checkpoint variable gets a handle (restored by the saver even if unused)
        for name in self.vals:
            self.var(name)
        return self


def export_bert_saved_model(export_dir, model, seq_len=128, tags=("serve",)):
    """SavedModel of a BERT masked-LM model: inputs ``input_ids`` / ``token_type_ids`` /
    ``input_mask`` (int32 ``[batch, seq_len]``), outputs ``sequence_output`` and the MLM
    ``mlm_logits`` / ``mlm_probabilities`` over every position."""
    _write_variables(export_dir, model)
    bg = _BertGraph(model, seq_len).build()
    _write_saved_model(export_dir, bg.g, bg.var_nodes, tags,
                       {k: (v, DT_INT32, [None, bg.S]) for k, v in bg.inputs.items()},
                       {k: (t, DT_FLOAT, dims) for k, (t, dims) in bg.outputs.items()})
    return export_dir
