"""Concrete optimizers with TF1-exact update math (see csrc/kernels/optim.hip header).

GPU: one fused HIP launch per contiguous region of the flat buffer (decayed / non-decayed) that
updates master weights, slots and the bf16 compute shadow together.
CPU: the same math in PyTorch (OneDeviceStrategy("/cpu:0"), BASELINE config 1).
"""
from __future__ import annotations

import math

import torch

from .base import FlatSlot, Optimizer, tf_adam_lr_t


def _K():
    from ..ops import native
    return native.kernels()


def _st():
    return torch.cuda.current_stream().cuda_stream


def _sh(space, start):
    return 0 if space.shadow is None else space.shadow.data_ptr() + start * space.shadow.element_size()


class GradientDescentOptimizer(Optimizer):
    """tf.train.GradientDescentOptimizer: p -= lr * g  (Momentum with mu = 0, no slot)."""

    def __init__(self, learning_rate, name="GradientDescent", **kw):
        super().__init__(learning_rate, name, **kw)

    def _build_slots(self):
        self._dummy = self.space.new_slot()

    def get_config(self):
        return {"type": "sgd", "learning_rate": self.learning_rate(),
                "weight_decay": self.weight_decay}

    def _apply_native(self, gscale):
        self._maybe_refresh_hyper()
        K, sp = _K(), self.space
        for s, e, dec in self._regions():
            K.sgd_momentum(sp.master.data_ptr() + 4 * s, sp.grad.data_ptr() + 4 * s,
                           self._dummy.data_ptr() + 4 * s, _sh(sp, s), e - s,
                           self._lr_dev.data_ptr(), 0.0, self.weight_decay if dec else 0.0,
                           gscale, 0, self._nonfinite.data_ptr(), _st())

    def _apply_reference(self, gscale):
        lr = self.learning_rate()
        sp = self.space
        with torch.no_grad():
            for s, e, dec in self._regions():
                g = sp.grad[s:e] * gscale + (self.weight_decay if dec else 0.0) * sp.master[s:e]
                sp.master[s:e].sub_(lr * g)


class MomentumOptimizer(Optimizer):
    """tf.train.MomentumOptimizer: a = mu*a + g; p -= lr*a (nesterov: p -= lr*(g + mu*a)).

    ``weight_decay`` adds the TF-official-ResNet L2 term (wd * p) to the gradient of decayed
    variables (everything except batch-norm parameters and biases)."""

    slot_names = ("Momentum",)

    def __init__(self, learning_rate, momentum=0.9, use_nesterov=False, name="Momentum", **kw):
        super().__init__(learning_rate, name, **kw)
        self.momentum = momentum
        self.use_nesterov = use_nesterov

    def _build_slots(self):
        self.slots = [FlatSlot("Momentum", self.space.new_slot())]

    def get_config(self):
        return {"type": "momentum", "learning_rate": self.learning_rate(),
                "momentum": self.momentum, "use_nesterov": self.use_nesterov,
                "weight_decay": self.weight_decay}

    def _apply_native(self, gscale):
        self._maybe_refresh_hyper()
        K, sp, a = _K(), self.space, self.slots[0].buf
        for s, e, dec in self._regions():
            K.sgd_momentum(sp.master.data_ptr() + 4 * s, sp.grad.data_ptr() + 4 * s,
                           a.data_ptr() + 4 * s, _sh(sp, s), e - s, self._lr_dev.data_ptr(),
                           float(self.momentum), self.weight_decay if dec else 0.0, gscale,
                           int(self.use_nesterov), self._nonfinite.data_ptr(), _st())

    def _apply_reference(self, gscale):
        lr, mu = self.learning_rate(), self.momentum
        sp, a = self.space, self.slots[0].buf
        with torch.no_grad():
            for s, e, dec in self._regions():
                g = sp.grad[s:e] * gscale + (self.weight_decay if dec else 0.0) * sp.master[s:e]
                a[s:e].mul_(mu).add_(g)
                step = g + mu * a[s:e] if self.use_nesterov else a[s:e]
                sp.master[s:e].sub_(lr * step)


SGD = MomentumOptimizer


class AdamOptimizer(Optimizer):
    """tf.train.AdamOptimizer with TF's epsilon placement:
    lr_t = lr*sqrt(1-b2^t)/(1-b1^t);  p -= lr_t * m / (sqrt(v) + eps)."""

    slot_names = ("Adam", "Adam_1")

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, name="Adam",
                 **kw):
        super().__init__(learning_rate, name, **kw)
        self.beta1, self.beta2, self.epsilon = beta1, beta2, epsilon

    def _build_slots(self):
        self.slots = [FlatSlot("Adam", self.space.new_slot()),
                      FlatSlot("Adam_1", self.space.new_slot())]

    def get_config(self):
        return {"type": "adam", "learning_rate": self.learning_rate(), "beta1": self.beta1,
                "beta2": self.beta2, "epsilon": self.epsilon}

    def lr_t(self):
        return tf_adam_lr_t(self.learning_rate(), self.beta1, self.beta2, self.iterations)

    def _refresh_hyper(self):
        self._lr_dev[0].fill_(self.lr_t())

    def _apply_native(self, gscale):
        self._maybe_refresh_hyper()
        K, sp = _K(), self.space
        m, v = self.slots[0].buf, self.slots[1].buf
        for s, e, dec in self._regions():
            K.adam(sp.master.data_ptr() + 4 * s, sp.grad.data_ptr() + 4 * s, m.data_ptr() + 4 * s,
                   v.data_ptr() + 4 * s, _sh(sp, s), e - s, self._lr_dev.data_ptr(),
                   float(self.beta1), float(self.beta2), float(self.epsilon),
                   self.weight_decay if dec else 0.0, gscale, self._nonfinite.data_ptr(), _st())

    def _apply_reference(self, gscale):
        lr_t = self.lr_t()
        sp = self.space
        m, v = self.slots[0].buf, self.slots[1].buf
        b1, b2 = self.beta1, self.beta2
        with torch.no_grad():
            for s, e, dec in self._regions():
                g = sp.grad[s:e] * gscale
                p = sp.master[s:e]
                m[s:e].mul_(b1).add_((1 - b1) * g)
                v[s:e].mul_(b2).add_((1 - b2) * g * g)
                wd = self.weight_decay if dec else 0.0
                p.sub_(lr_t * m[s:e] / (v[s:e].sqrt() + self.epsilon) + lr_t * wd * p)

    def non_slot_variables(self):
        # TF1 keeps the bias-correction powers as variables beta1_power / beta2_power
        t = self.iterations
        return {"beta1_power": torch.tensor(self.beta1 ** (t + 1)),
                "beta2_power": torch.tensor(self.beta2 ** (t + 1))}


class AdagradOptimizer(Optimizer):
    """tf.train.AdagradOptimizer: acc += g^2; p -= lr * g / sqrt(acc); acc0 = 0.1."""

    slot_names = ("Adagrad",)

    def __init__(self, learning_rate, initial_accumulator_value=0.1, name="Adagrad", **kw):
        super().__init__(learning_rate, name, **kw)
        self.initial_accumulator_value = initial_accumulator_value

    def _build_slots(self):
        self.slots = [FlatSlot("Adagrad", self.space.new_slot(self.initial_accumulator_value))]

    def get_config(self):
        return {"type": "adagrad", "learning_rate": self.learning_rate(),
                "initial_accumulator_value": self.initial_accumulator_value}

    def _apply_native(self, gscale):
        self._maybe_refresh_hyper()
        K, sp, acc = _K(), self.space, self.slots[0].buf
        for s, e, _ in self._regions():
            K.adagrad(sp.master.data_ptr() + 4 * s, sp.grad.data_ptr() + 4 * s,
                      acc.data_ptr() + 4 * s, _sh(sp, s), e - s, self._lr_dev.data_ptr(), gscale,
                      self._nonfinite.data_ptr(), _st())

    def _apply_reference(self, gscale):
        lr = self.learning_rate()
        sp, acc = self.space, self.slots[0].buf
        with torch.no_grad():
            for s, e, _ in self._regions():
                g = sp.grad[s:e] * gscale
                acc[s:e].add_(g * g)
                sp.master[s:e].sub_(lr * g * acc[s:e].rsqrt())


class LAMBOptimizer(Optimizer):
    """LAMB (layer-wise adaptive moments, You et al. 2019) for BERT pre-training
    (BASELINE.json config 5): per-variable trust ratio |p|/|u|."""

    slot_names = ("adam_m", "adam_v")     # google-research/bert optimization.py slot names
    elementwise = False

    def __init__(self, learning_rate, beta1=0.9, beta2=0.999, epsilon=1e-6, weight_decay=0.01,
                 name="LAMB", chunk=4096, **kw):
        super().__init__(learning_rate, name, weight_decay=weight_decay, **kw)
        self.beta1, self.beta2, self.epsilon, self.chunk = beta1, beta2, epsilon, chunk

    def get_config(self):
        return {"type": "lamb", "learning_rate": self.learning_rate(), "beta1": self.beta1,
                "beta2": self.beta2, "epsilon": self.epsilon, "weight_decay": self.weight_decay}

    def _build_slots(self):
        sp = self.space
        self.slots = [FlatSlot("adam_m", sp.new_slot()), FlatSlot("adam_v", sp.new_slot())]
        # chunk table {seg:int32, len:int32, start:int64} — one block per chunk
        rows = []
        wd = []
        for seg, (v, o) in enumerate(zip(sp.order, sp.offsets)):
            n = v.numel()
            wd.append(self.weight_decay if self.decay_filter(v) else 0.0)
            for c in range(0, n, self.chunk):
                rows.append((seg, min(self.chunk, n - c), o + c))
        self._nseg = len(sp.order)
        self._rows = rows
        self._tables = {}
        self._wd_seg = torch.tensor(wd, dtype=torch.float32, device=sp.device)
        self._norms = torch.zeros(2 * self._nseg, dtype=torch.float32, device=sp.device)
        self._hyper = torch.zeros(4, dtype=torch.float32, device=sp.device)

    def _chunk_table(self):
        """Chunk table for the whole space, or for the variables inside ``self._range`` (a
        colocated parameter-server shard; shard ranges fall on variable boundaries)."""
        key = getattr(self, "_range", None)
        if key not in self._tables:
            lo, hi = key if key is not None else (0, self.space.numel)
            rows = [r for r in self._rows if lo <= r[2] < hi]
            tbl = torch.zeros(max(1, len(rows)), 4, dtype=torch.int32)
            for i, (seg, ln, st) in enumerate(rows):
                tbl[i, 0], tbl[i, 1] = seg, ln
                tbl[i, 2], tbl[i, 3] = st & 0xFFFFFFFF if st < 2 ** 31 else st - 2 ** 32, st >> 32
            self._tables[key] = (tbl.to(self.space.device), len(rows))
        return self._tables[key]

    def _refresh_hyper(self):
        t = self.iterations
        self._hyper[0].fill_(1.0 / (1 - self.beta1 ** t))
        self._hyper[1].fill_(1.0 / (1 - self.beta2 ** t))
        self._lr_dev[0].fill_(self.learning_rate())

    def _apply_native(self, gscale):
        self._maybe_refresh_hyper()
        self._norms.zero_()
        sp, m, v = self.space, self.slots[0].buf, self.slots[1].buf
        chunks, nchunks = self._chunk_table()
        if nchunks == 0:
            return
        _K().lamb(sp.master.data_ptr(), sp.grad.data_ptr(), m.data_ptr(), v.data_ptr(),
                  _sh(sp, 0), chunks.data_ptr(), nchunks, self._hyper.data_ptr(),
                  self._lr_dev.data_ptr(), float(self.beta1), float(self.beta2),
                  float(self.epsilon), self._wd_seg.data_ptr(), gscale, self._norms.data_ptr(),
                  self._nonfinite.data_ptr(), _st())

    def _apply_reference(self, gscale):
        t = self.iterations
        lr = self.learning_rate()
        sp, m, v = self.space, self.slots[0].buf, self.slots[1].buf
        b1, b2 = self.beta1, self.beta2
        lo, hi = getattr(self, "_range", None) or (0, sp.numel)
        with torch.no_grad():
            for var, o in zip(sp.order, sp.offsets):
                if not lo <= o < hi:
                    continue
                n = var.numel()
                g = sp.grad[o:o + n] * gscale
                mm, vv, p = m[o:o + n], v[o:o + n], sp.master[o:o + n]
                mm.mul_(b1).add_((1 - b1) * g)
                vv.mul_(b2).add_((1 - b2) * g * g)
                wd = self.weight_decay if self.decay_filter(var) else 0.0
                u = (mm / (1 - b1 ** t)) / ((vv / (1 - b2 ** t)).sqrt() + self.epsilon) + wd * p
                pn, un = p.norm(), u.norm()
                trust = (pn / un) if (pn > 0 and un > 0) else 1.0
                p.sub_(lr * trust * u)


def clip_by_global_norm_(space, max_norm):
    """Scale the flat gradient buffer so that its global L2 norm <= max_norm; returns the norm."""
    if space.device.type == "cuda":
        out = torch.zeros(1, device=space.device, dtype=torch.float32)
        _K().sumsq(space.grad.data_ptr(), space.numel, out.data_ptr(), _st())
        norm = out.sqrt()
    else:
        norm = space.grad.norm().reshape(1)
    scale = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    space.grad.mul_(scale)
    return norm


def polynomial_decay(lr0, decay_steps, end_lr=0.0, power=1.0, warmup_steps=0):
    """tf.train.polynomial_decay with optional linear warm-up (BERT schedule)."""
    def f(step):
        if warmup_steps and step < warmup_steps:
            return lr0 * (step + 1) / warmup_steps
        s = min(step, decay_steps)
        return (lr0 - end_lr) * (1 - s / decay_steps) ** power + end_lr
    return f


def piecewise_constant(boundaries, values):
    def f(step):
        for b, v in zip(boundaries, values):
            if step < b:
                return v
        return values[-1]
    return f


def cosine_decay(lr0, decay_steps, alpha=0.0, warmup_steps=0):
    def f(step):
        if warmup_steps and step < warmup_steps:
            return lr0 * (step + 1) / warmup_steps
        s = min(step, decay_steps)
        return lr0 * ((1 - alpha) * 0.5 * (1 + math.cos(math.pi * s / decay_steps)) + alpha)
    return f
