"""SavedModel export (train/saved_model.py): decoded with an independent protobuf wire reader
and EXECUTED by a small TF-op interpreter written here, against the model's own forward.

TensorFlow is not importable (no network), so TF's loader cannot be run: instead this test does
what ``tf.compat.v1.saved_model.loader.load`` + a serving call do -- find the meta graph by tag,
run the SaverDef's restore op with the variables path fed to its filename tensor (RestoreV2 ->
AssignVariableOp per resource variable), then evaluate the ``serving_default`` signature's
outputs from its input -- with every op implemented from TF's documented semantics (NHWC,
SAME / EXPLICIT padding, FusedBatchNormV3 inference).  Parity with TF's own loader: unpinned.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from distributedtensorflow_amd.io import pbwire as pb
from distributedtensorflow_amd.io.bundle import BundleReader

DT = {1: np.float32, 3: np.int32}


def _attr(raw):
    a = pb.parse(raw)
    if 2 in a:
        return a[2][0].decode()
    if 3 in a:
        return a[3][0]
    if 4 in a:
        return pb.as_float(a[4][0])
    if 5 in a:
        return bool(a[5][0])
    if 6 in a:
        return ("type", a[6][0])
    if 7 in a:
        sh = pb.parse(a[7][0])
        return ("shape", [_signed(pb.parse(d).get(1, [0])[0]) for d in sh.get(2, [])])
    if 8 in a:
        return ("tensor", _tensor(a[8][0]))
    if 1 in a:
        lst = pb.parse(a[1][0])
        if 3 in lst:
            return [v for b in lst[3] for v in pb.unpack_varints(b)]
        if 6 in lst:
            return [v for b in lst[6] for v in pb.unpack_varints(b)]
        if 2 in lst:
            return [s.decode() for s in lst[2]]
        return []
    return None


def _signed(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def _tensor(raw):
    t = pb.parse(raw)
    dtype = t[1][0]
    dims = [_signed(pb.parse(d).get(1, [0])[0])
            for d in pb.parse(t[2][0]).get(2, [])] if 2 in t else []
    if dtype == 7:
        return np.array([s.decode() for s in t.get(8, [])], dtype=object).reshape(dims)
    return np.frombuffer(t[4][0], dtype=DT[dtype]).reshape(dims).copy()


def load_saved_model(export_dir):
    sm = pb.parse(open(os.path.join(export_dir, "saved_model.pb"), "rb").read())
    assert sm[1] == [1]
    meta = pb.parse(sm[2][0])
    info = pb.parse(meta[1][0])
    nodes = {}
    for nb in pb.parse(meta[2][0])[1]:
        n = pb.parse(nb)
        nodes[n[1][0].decode()] = {"op": n[2][0].decode(),
                                   "in": [i.decode() for i in n.get(3, [])],
                                   "attr": {k: _attr(v) for k, v in pb.parse_map(n.get(5, [])).items()}}
    saver = pb.parse(meta[3][0])
    sigs = {}
    for k, v in pb.parse_map(meta[5]).items():
        s = pb.parse(v)
        sigs[k] = {"inputs": {ik: pb.parse(iv)[1][0].decode() for ik, iv in pb.parse_map(s[1]).items()},
                   "outputs": {ok: pb.parse(ov)[1][0].decode() for ok, ov in pb.parse_map(s[2]).items()},
                   "method": s[3][0].decode()}
    return {"tags": [t.decode() for t in info.get(4, [])], "nodes": nodes,
            "saver": {"filename": saver[1][0].decode(), "restore": saver[3][0].decode(),
                      "version": saver[7][0]},
            "signatures": sigs}


class Interpreter:
    def __init__(self, graph):
        self.nodes = graph["nodes"]
        self.vars = {}

    def run(self, target, feed):
        memo = dict(feed)

        def ev(ref):
            if ref.startswith("^"):
                ev(ref[1:] + ":0")
                return None
            name, _, idx = ref.partition(":")
            idx = int(idx or 0)
            if (name, idx) in memo:
                return memo[(name, idx)]
            outs = self._op(name, ev)
            outs = outs if isinstance(outs, tuple) else (outs,)
            for i, o in enumerate(outs):
                memo[(name, i)] = o
            return memo[(name, idx)]
        return ev(target)

    def _op(self, name, ev):
        n = self.nodes[name]
        op, a = n["op"], n["attr"]
        ins = [ev(i) for i in n["in"] if not i.startswith("^")]
        for c in n["in"]:
            if c.startswith("^"):
                ev(c)
        t = torch.as_tensor
        if op == "Const":
            return a["value"][1]
        if op == "VarHandleOp":
            return a["shared_name"]
        if op == "ReadVariableOp":
            return self.vars[ins[0]]
        if op == "AssignVariableOp":
            self.vars[ins[0]] = ins[1]
            return None
        if op == "RestoreV2":
            r = BundleReader(str(ins[0].reshape(-1)[0]) if isinstance(ins[0], np.ndarray)
                             else ins[0])
            return tuple(r.get_tensor(nm) for nm in ins[1].reshape(-1))
        if op in ("Identity", "NoOp"):
            return ins[0] if ins else None
        if op == "Conv2D":
            x, w = t(ins[0]).permute(0, 3, 1, 2), t(ins[1]).permute(3, 2, 0, 1)
            s = a["strides"][1]
            kh, kw = w.shape[2], w.shape[3]
            if a["padding"] == "EXPLICIT":
                p = a["explicit_paddings"]
                x = F.pad(x, (p[4], p[5], p[2], p[3]))
            elif a["padding"] == "SAME":
                pads = []
                for dim, k in ((x.shape[3], kw), (x.shape[2], kh)):
                    out = -(-dim // s)
                    tot = max((out - 1) * s + k - dim, 0)
                    pads += [tot // 2, tot - tot // 2]
                x = F.pad(x, pads)
            return F.conv2d(x, w, stride=s).permute(0, 2, 3, 1).numpy()
        if op == "BiasAdd" or op == "AddV2":
            return ins[0] + ins[1]
        if op == "Relu":
            return np.maximum(ins[0], 0)
        if op == "FusedBatchNormV3":
            x, g, b, m, v = ins
            return (x - m) / np.sqrt(v + a["epsilon"]) * g + b
        if op == "PadV2":
            p = ins[1]
            return np.pad(ins[0], [tuple(r) for r in p], constant_values=float(ins[2]))
        if op == "MaxPool":
            k, s = a["ksize"][1], a["strides"][1]
            return F.max_pool2d(t(ins[0]).permute(0, 3, 1, 2), k, s).permute(0, 2, 3, 1).numpy()
        if op == "Mean":
            return ins[0].mean(axis=tuple(int(i) for i in np.reshape(ins[1], -1)),
                               keepdims=bool(a.get("keep_dims", False)))
        if op == "Reshape":
            return ins[0].reshape([int(s) for s in ins[1]])
        if op == "MatMul":
            x = ins[0].T if a.get("transpose_a") else ins[0]
            y = ins[1].T if a.get("transpose_b") else ins[1]
            return x @ y
        if op == "BatchMatMulV2":
            x = np.swapaxes(ins[0], -1, -2) if a.get("adj_x") else ins[0]
            y = np.swapaxes(ins[1], -1, -2) if a.get("adj_y") else ins[1]
            return np.matmul(x, y)
        if op == "GatherV2":
            return np.take(ins[0], ins[1], axis=int(ins[2]))
        if op == "Slice":
            begin, size = [int(v) for v in ins[1]], [int(v) for v in ins[2]]
            idx = tuple(slice(b, None if z == -1 else b + z) for b, z in zip(begin, size))
            return ins[0][idx]
        if op == "Transpose":
            return np.transpose(ins[0], [int(v) for v in ins[1]])
        if op == "Cast":
            return ins[0].astype(DT[a["DstT"][1]])
        if op == "Sub":
            return ins[0] - ins[1]
        if op == "Mul":
            return ins[0] * ins[1]
        if op == "SquaredDifference":
            return (ins[0] - ins[1]) ** 2
        if op == "Rsqrt":
            return 1.0 / np.sqrt(ins[0])
        if op == "Pow":
            return np.power(ins[0], ins[1])
        if op == "Tanh":
            return np.tanh(ins[0])
        if op == "Softmax":
            e = np.exp(ins[0] - ins[0].max(-1, keepdims=True))
            return e / e.sum(-1, keepdims=True)
        if op == "Placeholder":
            raise KeyError(f"placeholder {name} not fed")
        raise NotImplementedError(op)


def _serve(export_dir, x):
    g = load_saved_model(export_dir)
    assert "serve" in g["tags"] and g["saver"]["version"] == 2
    it = Interpreter(g)
    prefix = os.path.join(export_dir, "variables", "variables")
    fname, _, _ = g["saver"]["filename"].partition(":")
    it.run("^" + g["saver"]["restore"], {(fname, 0): np.array([prefix], dtype=object)})
    sig = g["signatures"]["serving_default"]
    assert sig["method"] == "tensorflow/serving/predict"
    inp = sig["inputs"]["images"].split(":")[0]
    feed = {(inp, 0): x}
    return g, it, it.run(sig["outputs"]["logits"], feed), it.run(sig["outputs"]["probabilities"],
                                                                 feed)


@pytest.mark.parametrize("kind", ["mnist_cnn", "mnist_mlp", "resnet50"])
def test_saved_model_graph_serves_like_the_model(tmp_path, kind):
    from distributedtensorflow_amd.models import MnistCNN, MnistMLP, resnet50
    from distributedtensorflow_amd.train import save_saved_model
    torch.manual_seed(0)
    model = {"mnist_cnn": MnistCNN, "mnist_mlp": MnistMLP, "resnet50": resnet50}[kind]()
    with torch.no_grad():
        for m in model.modules():          # non-trivial moving statistics for the BN check
            if hasattr(m, "moving_mean"):
                m.moving_mean.uniform_(-0.2, 0.2)
                m.moving_variance.uniform_(0.5, 2.0)
    model.eval()
    shape = (2, 784) if kind != "resnet50" else (1, 224, 224, 3)
    x = torch.randn(*shape)
    with torch.no_grad():
        want = model(x).float().numpy()
    exp = save_saved_model(str(tmp_path / "export"), model)
    g, it, logits, probs = _serve(exp, x.numpy())
    # every checkpoint variable was restored through the graph's saver
    keys = set(BundleReader(os.path.join(exp, "variables", "variables")).keys()) - {""}
    assert set(it.vars) == keys
    np.testing.assert_allclose(logits, want, rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(probs.sum(-1), 1.0, rtol=1e-5)
    ops_used = {n["op"] for n in g["nodes"].values()}
    assert {"VarHandleOp", "ReadVariableOp", "RestoreV2", "SaveV2", "AssignVariableOp",
            "MatMul"} <= ops_used
    if kind == "resnet50":
        assert {"Conv2D", "FusedBatchNormV3", "MaxPool", "PadV2", "Mean", "AddV2"} <= ops_used


def test_bert_saved_model_serves_like_the_model(tmp_path):
    """a 2-layer BERT MLM model exported as a SavedModel (stock TF ops for the
    fused training kernels: GatherV2 embeddings, moments LayerNorm, BatchMatMulV2 attention with
    the -10000 key mask, tanh-GELU, tied decoder MatMul) executes in the independent
    interpreter and reproduces the model's own inference logits at every position."""
    from distributedtensorflow_amd.models.bert import BertConfig, BertForPreTraining
    from distributedtensorflow_amd.train import save_saved_model
    torch.manual_seed(0)
    cfg = BertConfig(vocab_size=120, hidden_size=128, num_hidden_layers=2,
                     num_attention_heads=2, intermediate_size=256, max_position_embeddings=64)
    model = BertForPreTraining(cfg)
    with torch.no_grad():               # non-trivial LN / bias parameters
        for n, p in model.named_parameters():
            if p.dim() == 1:
                p.add_(0.1 * torch.randn_like(p))
    model.eval()
    B, S = 3, 16
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (B, S), generator=g)
    tt = torch.randint(0, 2, (B, S), generator=g)
    mask = torch.ones(B, S, dtype=torch.int64)
    mask[1, 11:] = 0
    mask[2, 5:] = 0
    with torch.no_grad():
        want = model(ids, tt, mask).float().reshape(B, S, -1).numpy()
    exp = save_saved_model(str(tmp_path / "bert"), model, seq_len=S)
    graph = load_saved_model(exp)
    it = Interpreter(graph)
    prefix = os.path.join(exp, "variables", "variables")
    fname, _, _ = graph["saver"]["filename"].partition(":")
    it.run("^" + graph["saver"]["restore"], {(fname, 0): np.array([prefix], dtype=object)})
    keys = set(BundleReader(prefix).keys()) - {""}
    assert set(it.vars) == keys
    sig = graph["signatures"]["serving_default"]
    assert set(sig["inputs"]) == {"input_ids", "token_type_ids", "input_mask"}
    feed = {(sig["inputs"][k].split(":")[0], 0): v.numpy().astype(np.int32)
            for k, v in (("input_ids", ids), ("token_type_ids", tt), ("input_mask", mask))}
    logits = it.run(sig["outputs"]["mlm_logits"], feed)
    assert logits.shape == (B, S, cfg.vocab_size)
    np.testing.assert_allclose(logits, want, rtol=2e-3, atol=2e-3)
    seq = it.run(sig["outputs"]["sequence_output"], feed)
    assert seq.shape == (B, S, cfg.hidden_size)
    probs = it.run(sig["outputs"]["mlm_probabilities"], feed)
    np.testing.assert_allclose(probs.sum(-1), 1.0, rtol=1e-5)
    ops_used = {n["op"] for n in graph["nodes"].values()}
    assert {"GatherV2", "BatchMatMulV2", "Softmax", "Tanh", "Rsqrt", "SquaredDifference",
            "Transpose", "MatMul", "BiasAdd"} <= ops_used
    # TF checkpoint names of modeling.py (query/key/value split out of the fused QKV kernel)
    assert "bert/encoder/layer_1/attention/self/key/kernel" in keys
    assert graph["nodes"]["cls/predictions/MatMul"]["attr"]["transpose_b"] is True
