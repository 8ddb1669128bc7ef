"""``tf.train.Saver`` with the TF checkpoint-V2 on-disk layout.

Files for ``save(..., "model.ckpt", global_step=N)``:
  * ``model.ckpt-N.index`` / ``model.ckpt-N.data-00000-of-00001`` — tensor bundle (native C++);
  * ``model.ckpt-N.meta`` — a minimal MetaGraphDef (meta_info_def + saver_def; no graph);
  * ``checkpoint`` — the CheckpointState text proto (``model_checkpoint_path``,
    ``all_model_checkpoint_paths``, timestamps), pruned to ``max_to_keep``.
Keys and layouts are TF's: ``conv2d/kernel`` is stored HWIO (internally KRSC), dense kernels
``[in, out]`` (internally ``[out, in]``), Adam slots ``<var>/Adam``, ``<var>/Adam_1`` plus
``beta1_power``/``beta2_power``, Momentum ``<var>/Momentum``, and ``global_step`` (int64).
"""
from __future__ import annotations

import glob
import os
import re
import time

import numpy as np
import torch

from ..io.bundle import BundleReader, write_bundle


# ----------------------------------------------------------------------------- layouts

def to_tf_layout(t: torch.Tensor, layout):
    if layout == "KRSC":           # [K,R,S,C] -> HWIO [R,S,C,K]
        return t.permute(1, 2, 3, 0)
    if layout == "OI":             # [out,in] -> [in,out]
        return t.t()
    return t


def from_tf_layout(a: np.ndarray, layout):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if layout == "KRSC":
        return t.permute(3, 0, 1, 2)
    if layout == "OI":
        return t.t()
    return t


def collect_checkpoint_vars(model=None, optimizer=None, global_step=None, strategy=None):
    """{tf_name: (tensor, layout)} for a model (+ optimizer slots, global step)."""
    from ..models.layers import collect_variables
    out = {}
    layouts = {}
    if model is not None:
        for name, t, layout in collect_variables(model):
            out[name] = t
            layouts[name] = layout
    if optimizer is not None and optimizer.space is not None:
        for name, t in optimizer.slot_variables().items():
            base = name.rsplit("/", 1)[0]
            out[name] = t
            layouts[name] = layouts.get(base)
        for name, t in optimizer.non_slot_variables().items():
            out[name] = t
            layouts[name] = None
    if global_step is not None:
        gs_t = global_step.tensor if hasattr(global_step, "tensor") else global_step
        out["global_step"] = gs_t
        layouts["global_step"] = None
    return {k: (v, layouts.get(k)) for k, v in out.items()}


# ----------------------------------------------------------------------------- state file

def _state_path(d):
    return os.path.join(d, "checkpoint")


def update_checkpoint_state(save_dir, model_checkpoint_path, all_paths, timestamps=None):
    lines = [f'model_checkpoint_path: "{model_checkpoint_path}"']
    lines += [f'all_model_checkpoint_paths: "{p}"' for p in all_paths]
    if timestamps:
        lines += [f"all_model_checkpoint_timestamps: {t:.6f}" for t in timestamps]
        lines.append(f"last_preserved_timestamp: {timestamps[-1]:.6f}")
    tmp = _state_path(save_dir) + ".tmp"
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, _state_path(save_dir))


class CheckpointState:
    def __init__(self, model_checkpoint_path, all_model_checkpoint_paths, timestamps=()):
        self.model_checkpoint_path = model_checkpoint_path
        self.all_model_checkpoint_paths = list(all_model_checkpoint_paths)
        self.all_model_checkpoint_timestamps = list(timestamps)


def get_checkpoint_state(checkpoint_dir):
    p = _state_path(checkpoint_dir)
    if not os.path.exists(p):
        return None
    model, alls, ts = None, [], []
    with open(p) as f:
        for line in f:
            m = re.match(r'\s*(\w+):\s*"?(.*?)"?\s*$', line)
            if not m:
                continue
            k, v = m.group(1), m.group(2)
            if k == "model_checkpoint_path":
                model = v
            elif k == "all_model_checkpoint_paths":
                alls.append(v)
            elif k == "all_model_checkpoint_timestamps":
                ts.append(float(v))

    def absolutize(x):
        return x if os.path.isabs(x) else os.path.join(checkpoint_dir, x)
    return CheckpointState(absolutize(model) if model else None, [absolutize(a) for a in alls], ts)


def latest_checkpoint(checkpoint_dir):
    st = get_checkpoint_state(checkpoint_dir)
    if st is None or not st.model_checkpoint_path:
        return None
    if os.path.exists(st.model_checkpoint_path + ".index"):
        return st.model_checkpoint_path
    return None


def checkpoint_exists(prefix):
    return os.path.exists(prefix + ".index")


# ----------------------------------------------------------------------------- meta graph

def _pb_str(field, s):
    b = s.encode()
    return _varint((field << 3) | 2) + _varint(len(b)) + b


def _pb_int(field, v):
    return _varint(field << 3) + _varint(v)


def _pb_msg(field, body: bytes):
    return _varint((field << 3) | 2) + _varint(len(body)) + body


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def meta_graph_bytes(var_names, max_to_keep=5):
    meta_info = _pb_str(1, "dtf-v1") + _pb_str(5, "1.15.0-dtf")
    saver_def = (_pb_str(1, "save/Const:0") + _pb_str(2, "save/control_dependency:0") +
                 _pb_str(3, "save/restore_all") + _pb_int(4, max_to_keep) + _pb_int(7, 2))
    collection = b"".join(_pb_str(1, n) for n in var_names)      # informational
    return _pb_msg(1, meta_info) + _pb_msg(2, b"") + _pb_msg(3, saver_def) + \
        _pb_msg(4, _pb_str(1, "variables") + _pb_msg(2, _pb_msg(2, collection)))


# ----------------------------------------------------------------------------- Saver

class Saver:
    """tf.train.Saver.  ``var_list``: dict ``{tf_name: tensor}`` / ``{tf_name: (tensor, layout)}``,
    or a model (its variables), or None with ``model=/optimizer=/global_step=``."""

    def __init__(self, var_list=None, max_to_keep=5, model=None, optimizer=None,
                 global_step=None, write_meta_graph=True, num_shards=1):
        self._var_list = var_list
        self.model, self.optimizer, self.global_step = model, optimizer, global_step
        self.max_to_keep = max_to_keep
        self.write_meta_graph = write_meta_graph
        self.num_shards = num_shards
        self._last = []    # [(prefix, timestamp)]

    def _vars(self):
        if self._var_list is None:
            return collect_checkpoint_vars(self.model, self.optimizer, self.global_step)
        if isinstance(self._var_list, torch.nn.Module):
            return collect_checkpoint_vars(self._var_list)
        out = {}
        for k, v in self._var_list.items():
            out[k] = v if isinstance(v, tuple) else (v, getattr(v, "_dtf_layout", None))
        return out

    def save(self, sess=None, save_path="model.ckpt", global_step=None, write_meta_graph=None,
             values=None):
        """Returns the checkpoint prefix.  ``values`` optionally overrides tensor contents
        (e.g. gathered from parameter-server shards)."""
        if global_step is not None:
            step = int(global_step) if not hasattr(global_step, "value") else global_step.value()
            prefix = f"{save_path}-{step}"
        else:
            prefix = save_path
        d = os.path.dirname(os.path.abspath(prefix))
        os.makedirs(d, exist_ok=True)
        if self.optimizer is not None and getattr(self.optimizer, "space", None) is not None:
            self.optimizer.synchronize_variables()    # overlapped parameter-server gathers
        tensors = {}
        for name, (t, layout) in self._vars().items():
            if values is not None and name in values:
                t = values[name]
            t = t.detach() if isinstance(t, torch.Tensor) else torch.as_tensor(t)
            tensors[name] = to_tf_layout(t.cpu(), layout).contiguous()
        # the copies above waited for the step's collectives: if the watchdog aborted one of
        # them (dead peer), these values are garbage -- never let them become the latest
        # checkpoint that recovery restores
        from ..parallel import watchdog
        watchdog.check()
        if self.num_shards > 1:
            names = sorted(tensors)
            write_bundle(prefix, tensors, self.num_shards,
                         lambda n: names.index(n) % self.num_shards)
        else:
            write_bundle(prefix, tensors)
        wm = self.write_meta_graph if write_meta_graph is None else write_meta_graph
        if wm:
            with open(prefix + ".meta", "wb") as f:
                f.write(meta_graph_bytes(sorted(tensors), self.max_to_keep))
        now = time.time()
        self._last = [(p, t) for p, t in self._last if p != prefix] + [(prefix, now)]
        if self.max_to_keep and len(self._last) > self.max_to_keep:
            for old, _ in self._last[:-self.max_to_keep]:
                for f in glob.glob(old + ".*"):
                    os.remove(f)
            self._last = self._last[-self.max_to_keep:]
        update_checkpoint_state(d, os.path.basename(prefix),
                                [os.path.basename(p) for p, _ in self._last],
                                [t for _, t in self._last])
        return prefix

    def restore(self, sess=None, save_path=None, strict=True):
        reader = BundleReader(save_path)
        have = set(reader.keys())
        missing = []
        with torch.no_grad():
            for name, (t, layout) in self._vars().items():
                if name not in have:
                    missing.append(name)
                    continue
                val = from_tf_layout(reader.get_tensor(name), layout)
                if name == "global_step" and self.global_step is not None and \
                        hasattr(self.global_step, "assign"):
                    self.global_step.assign(int(val.reshape(-1)[0]))
                    continue
                if isinstance(t, torch.Tensor):
                    t.copy_(val.to(t.dtype).reshape(t.shape))
                    sh = getattr(t, "_dtf_shadow", None)
                    if sh is not None:
                        sh.copy_(t)
        if self.optimizer is not None and "beta1_power" in have and \
                hasattr(self.optimizer, "beta1"):
            b1p = float(reader.get_tensor("beta1_power"))
            self.optimizer.iterations = max(0, int(round(np.log(b1p) /
                                                         np.log(self.optimizer.beta1))) - 1)
        if strict and missing:
            raise KeyError(f"variables not found in checkpoint {save_path}: {missing[:8]}")
        return missing

    @property
    def last_checkpoints(self):
        return [p for p, _ in self._last]


def list_variables(ckpt):
    if os.path.isdir(ckpt):
        ckpt = latest_checkpoint(ckpt)
    r = BundleReader(ckpt)
    return [(k, r.entry(k)["shape"]) for k in sorted(r.keys())]


def load_variable(ckpt, name):
    if os.path.isdir(ckpt):
        ckpt = latest_checkpoint(ckpt)
    return BundleReader(ckpt).get_tensor(name)


# ----------------------------------------------------------------------------- SavedModel

def save_saved_model(export_dir, model, tags=("serve",), input_shape=None, seq_len=128):
    """SavedModel directory: ``saved_model.pb`` (inference GraphDef traced from the model, the
    saver subgraph and a ``serving_default`` signature; train/saved_model.py) +
    ``variables/variables.{index,data-00000-of-00001}``.  ``input_shape`` defaults to the
    model's ``input_signature_shape`` (``None`` = the batch dimension).  BERT models export
    their own graph (token-id inputs of length ``seq_len``)."""
    from .saved_model import export_bert_saved_model, export_saved_model
    from ..models.bert import BertForPreTraining
    if isinstance(model, BertForPreTraining):
        return export_bert_saved_model(export_dir, model, seq_len, tags)
    shape = input_shape or getattr(model, "input_signature_shape", None)
    if shape is None:
        raise ValueError("save_saved_model needs input_shape= for this model")
    return export_saved_model(export_dir, model, tuple(shape), tags)


def load_saved_model_variables(export_dir, model):
    saver = Saver(model)
    return saver.restore(save_path=os.path.join(export_dir, "variables", "variables"))
