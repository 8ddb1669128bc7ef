"""Optimizer base: TF1-style ``minimize / compute_gradients / apply_gradients`` on flat buffers.

Reference usage: ``tf.train.AdamOptimizer(5e-4).minimize(loss,
global_step=global_step)`` (``run_mnist_distributed.py:116``), Adam 0.01
(``templates/00_mnist_replica.py:166``), Adagrad 0.01 (``templates/00_between…:34``).

MI355X design: on first use every trainable variable is re-homed into ONE flat fp32 master
buffer (views), gradients live in ONE flat fp32 buffer (views; autograd accumulates into them in
place) and each optimizer slot is one flat buffer.  The update is therefore a single fused HIP
launch over the whole model (no per-tensor launches, no multi-tensor lists), and the strategy's
gradient all-reduce operates on contiguous bucket slices of the same flat gradient buffer.

Layout: variables are placed in REVERSE creation order (backward produces gradients roughly
last-layer-first, so contiguous buckets complete in order), decayed variables first, then the
non-decayed ones (BatchNorm gamma/beta, biases) in their own tail region.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass

import torch

from ..train import global_step as gs


@dataclass
class FlatSlot:
    name: str           # TF slot suffix, e.g. "Momentum", "Adam", "Adam_1"
    buf: torch.Tensor


class FlatSpace:
    """Owns the flat master / grad / shadow buffers of a set of variables."""

    def __init__(self, variables, decay_filter=None, shadow_dtype=None, align=64):
        variables = [v for v in variables if v.requires_grad]
        if not variables:
            raise ValueError("no trainable variables")
        dev = variables[0].device
        decay_filter = decay_filter or (lambda v: True)
        decayed = [v for v in reversed(variables) if decay_filter(v)]
        plain = [v for v in reversed(variables) if not decay_filter(v)]
        self.order = decayed + plain
        self.offsets = []
        off = 0
        for v in self.order:
            self.offsets.append(off)
            off += -(-v.numel() // align) * align   # keep every view 256-B aligned
        self.n_decay = -(-sum(v.numel() for v in decayed) // 1)
        self.decay_end = self.offsets[len(decayed)] if plain else off
        self.numel = off
        self.device = dev
        self.master = torch.zeros(off, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(off, device=dev, dtype=torch.float32)
        self.shadow = (torch.zeros(off, device=dev, dtype=shadow_dtype)
                       if shadow_dtype is not None else None)
        with torch.no_grad():
            for v, o in zip(self.order, self.offsets):
                n = v.numel()
                self.master[o:o + n].copy_(v.detach().reshape(-1).float())
                v.data = self.master[o:o + n].view(v.shape)
                v.grad = self.grad[o:o + n].view(v.shape)
                v._dtf_flat = True           # kernels may accumulate into v.grad directly
                v._dtf_grad_ready = None     # set by gradient-bucketing reducers
                if self.shadow is not None:
                    s = self.shadow[o:o + n].view(v.shape)
                    s.copy_(v.data)
                    v._dtf_shadow = s
        self.index = {id(v): i for i, v in enumerate(self.order)}

    def zero_grad(self):
        self.grad.zero_()

    def refresh_shadow(self):
        if self.shadow is not None:
            self.shadow.copy_(self.master)

    def new_slot(self, fill=0.0):
        return torch.full((self.numel,), float(fill), device=self.device, dtype=torch.float32)

    def view_of(self, buf, v):
        i = self.index[id(v)]
        o = self.offsets[i]
        return buf[o:o + v.numel()].view(v.shape)

    def regions(self):
        """[(start, end, decayed)] contiguous regions of the flat buffer."""
        out = [(0, self.decay_end, True)]
        if self.decay_end < self.numel:
            out.append((self.decay_end, self.numel, False))
        return [r for r in out if r[1] > r[0]]


def default_decay_filter(v):
    """TF official ResNet convention: L2 on everything but batch-norm variables and biases."""
    name = getattr(v, "_dtf_name", "")
    return not (re.search(r"(batch_norm|_bn/|/gamma|/beta|/bias)", name) or v.dim() <= 1)


class Optimizer:
    """Base class.  Subclasses implement ``_build_slots`` and ``_apply_native/_apply_reference``."""

    slot_names: tuple = ()
    # the update of each element depends only on that element's gradient / slots (a sharded
    # parameter server may then split variables between owners); LAMB's per-tensor trust ratio
    # is not elementwise
    elementwise: bool = True

    def __init__(self, learning_rate, name, weight_decay=0.0, decay_filter=None,
                 use_locking=False):
        self._lr_value = learning_rate
        self.name = name
        self.weight_decay = weight_decay
        self.decay_filter = decay_filter or default_decay_filter
        self.space: FlatSpace | None = None
        self.slots: list[FlatSlot] = []
        self.iterations = 0          # number of applied updates (TF: beta powers / global step)
        self._lr_dev = None
        self._nonfinite = None
        self._reducer = None
        self.use_locking = use_locking
        # bf16 compute shadow of the fp32 masters ("auto": on GPUs); None for fp32-compute models
        self.shadow_dtype = "auto"
        # True while a training step is being captured into a HIP graph (train/graphed.py): the
        # per-step hyper-parameters are then written by the replay wrapper, not by the step
        self._capturing = False

    # ------------------------------------------------------------------ hyper-parameters
    def learning_rate(self, step=None):
        lr = self._lr_value
        return float(lr(step if step is not None else self.iterations)) if callable(lr) else float(lr)

    # ------------------------------------------------------------------ build
    def build(self, variables):
        if self.space is not None:
            return self.space
        from ..parallel import strategy as _strat
        variables = list(variables)
        dev = variables[0].device
        shadow = (torch.bfloat16 if dev.type == "cuda" else None) if self.shadow_dtype == "auto" \
            else self.shadow_dtype
        self.space = FlatSpace(variables, self.decay_filter, shadow)
        self.space.elementwise = self.elementwise      # read by sharding gradient reducers
        self._build_slots()
        self._lr_dev = torch.zeros(4, device=dev, dtype=torch.float32)
        self._nonfinite = torch.zeros(1, device=dev, dtype=torch.int32)
        strat = _strat.get_strategy()
        self._reducer = strat.make_gradient_reducer(self.space)
        strat.broadcast_space(self.space)
        return self.space

    def _build_slots(self):
        raise NotImplementedError

    # ------------------------------------------------------------------ TF1 API
    def compute_gradients(self, loss, var_list=None):
        if self.space is None:
            self.build(var_list)
        from .. import profiler
        self.space.zero_grad()
        self._reducer.begin_step()
        fn = getattr(loss, "grad_fn", None)
        if fn is not None and getattr(fn, "dtf_unit_grad_ok", False):
            fn.dtf_unit_grad = True          # backward() below seeds exactly d(loss) = 1
        with profiler.maybe_phase("backward"):
            loss.backward()
        # every deferred-work record of this step has been consumed (or never will be)
        from .. import ops
        ops.end_step()
        with profiler.maybe_phase("comm"):
            self._reducer.finish()
        return [(v.grad, v) for v in self.space.order]

    def apply_gradients(self, grads_and_vars=None, global_step=None):
        assert self.space is not None, "call build()/compute_gradients() first"
        self.iterations += 1
        if getattr(self._reducer, "applies_update", False):
            # parameter-server strategies: the PS owning the variables applies the update
            step = self._reducer.apply_remote(self)
            if global_step is not None:
                if step is None:                 # colocated owners: a local synchronous step
                    gs.increment(global_step)
                elif hasattr(global_step, "assign"):
                    global_step.assign(step)     # the PS's authoritative global step
            return step
        from .. import profiler
        with profiler.maybe_phase("optimizer"):
            self._apply(self._reducer.grad_scale())
        if global_step is not None:
            gs.increment(global_step)
        return None

    def get_config(self) -> dict:
        """Serializable description (shipped to parameter-server tasks)."""
        raise NotImplementedError

    def minimize(self, loss, global_step=None, var_list=None):
        """backward -> (cross-replica reduce, overlapped) -> fused update -> global_step += 1."""
        if var_list is None:
            var_list = _infer_vars(loss)
        self.compute_gradients(loss, var_list)
        return self.apply_gradients(None, global_step)

    # ------------------------------------------------------------------ update
    def _refresh_hyper(self):
        """Write this step's hyper-parameters into the device buffers the fused kernels read
        (learning rate; Adam's lr_t; LAMB's bias corrections)."""
        self._lr_dev[0].fill_(self.learning_rate())

    def _maybe_refresh_hyper(self):
        # inside a graph capture the fill would be recorded with THIS step's constant; the
        # replay wrapper refreshes the buffers before every replay instead
        if not self._capturing:
            self._refresh_hyper()

    def _apply(self, gscale, rng=None):
        """Run the update over the whole flat buffer, or only over ``rng = (start, end)`` (the
        slice a parameter-server shard owns)."""
        self._range = rng
        try:
            if self.space.device.type == "cuda":
                self._apply_native(gscale)
            else:
                self._apply_reference(gscale)
        finally:
            self._range = None

    def _regions(self):
        regs = self.space.regions()
        rng = getattr(self, "_range", None)
        if rng is None:
            return regs
        lo, hi = rng
        return [(max(s, lo), min(e, hi), d) for s, e, d in regs if min(e, hi) > max(s, lo)]

    def synchronize_variables(self):
        """Wait for communication still writing the variables (a colocated parameter server
        gathers updated shards overlapped with the next forward); call before reading the
        master weights outside a training step (checkpoint, replica check, evaluation)."""
        if self._reducer is not None:
            self._reducer.drain()

    def gather_state(self):
        """Collective: complete every optimizer slot on every rank (a sharded parameter server
        keeps each slot slice only on its owner) -- before a checkpoint of the slots."""
        if self._reducer is not None:
            self._reducer.gather_state(self.state_tensors())

    def nonfinite_flag(self):
        return bool(self._nonfinite.item()) if self._nonfinite is not None else False

    def slot_variables(self):
        """{tf_name: tensor view} for checkpointing (e.g. 'conv2d/kernel/Adam')."""
        out = {}
        for slot in self.slots:
            for v in self.space.order:
                view = self.space.view_of(slot.buf, v)
                splits = getattr(v, "_dtf_splits", None)   # fused variables (e.g. BERT Q|K|V)
                if splits:
                    for name, s, e in splits:
                        out[f"{name}/{slot.name}"] = view[s:e]
                else:
                    out[f"{v._dtf_name}/{slot.name}"] = view
        return out

    def non_slot_variables(self):
        return {}

    def state_tensors(self):
        return [s.buf for s in self.slots]


def _infer_vars(loss):
    """Collect leaf parameters reachable from ``loss`` (TF: trainable_variables of the graph)."""
    seen, out, stack = set(), [], [loss.grad_fn]
    while stack:
        fn = stack.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        if hasattr(fn, "variable"):
            out.append(fn.variable)
        for nxt, _ in fn.next_functions:
            stack.append(nxt)
    out.reverse()
    return out


def tf_adam_lr_t(lr, beta1, beta2, t):
    return lr * math.sqrt(1.0 - beta2 ** t) / (1.0 - beta1 ** t)
