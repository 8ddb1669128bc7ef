"""Deferred-work records: the cross-op hand-offs of the native op layer, in one place.

Several fused paths leave work for a LATER op instead of running a pass of their own
(``ops/native.py``):

* :class:`BnDeferred` -- a BatchNorm + ReLU output whose apply pass never ran: the consuming 3x3
  conv normalises its input on load (``y._dtf_bnl``);
* :class:`Recompute` -- a bottleneck c3 output that was never stored: its readers recompute it
  from the conv's input and weight (``out._dtf_recompute``);
* :class:`LazyBnDx` -- the d(x) of a residual BatchNorm not yet formed: the fused c3 backward
  forms it per tile (handed over through a :class:`GradSlot`, ``out._dtf_lazy_slot``);
* :class:`MaskedGrad` -- a residual gradient kept as (dy, ReLU bit mask): the dgrad epilogue of
  the conv that also reads the residual adds it (``x._dtf_pending_grad`` / a grad slot);
* :class:`LazyStemDz` -- the ResNet stem conv's output gradient (BN + ReLU + max-pool backward)
  not yet formed: the stem weight gradient forms it on load (``out._dtf_stem_slot``).

These records ride on activation tensors, so their lifetime is the activations'.  Round 5 found
what that costs when it goes wrong: a y <-> record reference cycle left every step's c1 outputs
to Python's cyclic collector (+2.9 GB of peak memory per ResNet-50 step,
profiles/measurements/r5_bnl_reference_cycle_fix.jsonl).  The lifetime rule, enforced here for
every kind:

1. a record never holds a strong reference to the tensor it is attached to (``weakref``);
2. every record registers with the step registry when created, and :func:`end_step` -- called by
   ``Optimizer.compute_gradients`` once the backward pass has returned -- RELEASES every record
   still alive: its operand references are dropped (which also breaks the one hand-off that is a
   cycle by construction while it waits: c3's output -> its grad slot -> LazyBnDx -> that output)
   and any later use raises instead of reading a finished step's buffers.

So no record outlives the step that made it, whether or not its consumer ran
(tests/test_native_records.py: CPU; tests/test_resnet_gpu.py: peak memory flat over 25 steps).
Plain Python objects: importable without the HIP extension (kernels are reached lazily).
"""
from __future__ import annotations

import weakref

_LIVE = weakref.WeakSet()          # records created since the last end_step()


class ReleasedRecordError(RuntimeError):
    """A deferred-work record was used after the step that created it ended."""


class _Record:
    __slots__ = ("released", "__weakref__")

    def __init__(self):
        self.released = False
        _LIVE.add(self)

    def _check(self):
        if self.released:
            raise ReleasedRecordError(
                f"{type(self).__name__} used after its training step ended (records are "
                "released by ops.end_step(), called after every backward)")

    def release(self):
        """Drop every operand reference (idempotent)."""
        for name in type(self).__slots__:
            setattr(self, name, None)
        self.released = True


def _native():
    from . import native
    return native


class BnDeferred(_Record):
    """A BatchNorm + ReLU output whose apply pass has not run (``batch_norm(..., defer=True)``):
    the consuming 3x3 conv normalises its input on load and writes ``y`` itself (halo kernels,
    csrc/kernels/conv.hip BNL); any other use materialises it first with the apply pass."""
    __slots__ = ("x", "scale", "shift", "y", "done")

    def __init__(self, x, scale, shift, y):
        super().__init__()
        # y holds this record: a weak reference back (rule 1)
        self.x, self.scale, self.shift, self.y, self.done = x, scale, shift, weakref.ref(y), False

    def release(self):
        super().release()
        self.done = True                     # nothing pending: a released record is inert

    def materialize(self):
        self._check()
        y = self.y()
        if not self.done and y is not None:
            n = _native()
            C = self.x.shape[-1]
            n._K.bn_apply(self.x.data_ptr(), 0, y.data_ptr(), self.scale.data_ptr(),
                          self.shift.data_ptr(), self.x.numel() // C, C, 1, n._st(), 0)
            self.done = True
        return y


class Recompute(_Record):
    """A bottleneck c3 output that was never stored (lazy x3): x3 = bf16(y . w^T) with y the
    conv's input [M, K3] and w its bf16 weight [N, K3, ...] -- recomputed with the producing
    stream GEMM's exact MFMA chain by the residual BN's apply (gemm_stream_apply), by the
    consuming data gradient's BN-sum epilogue (gemm_stream_bnb RC) and by the fused c3 backward
    (RC); :meth:`materialize` writes it into the tensor's own storage for any other reader."""
    __slots__ = ("y", "wb", "out", "done")

    def __init__(self, y, wb, out):
        super().__init__()
        # the output holds this record: a weak reference back (rule 1)
        self.y, self.wb, self.out, self.done = y, wb, weakref.ref(out), False

    @property
    def k3(self):
        self._check()
        return self.y.shape[-1]

    def materialize(self):
        self._check()
        out = self.out()
        if not self.done and out is not None:
            N = out.shape[-1]
            M = out.numel() // N
            _native().gemm_nt(self.y.view(M, self.k3), self.wb.view(N, self.k3),
                              out=out.view(M, N))
            self.done = True
        return out


class MaskedGrad(_Record):
    """d(residual) of a residual+ReLU BatchNorm kept as (dy, forward ReLU bit mask) rather
    than a materialised bf16 tensor; the identity-shortcut dgrad adds dy * mask in its
    epilogue."""
    __slots__ = ("dy", "mask")

    def __init__(self, dy, mask):
        super().__init__()
        self.dy, self.mask = dy, mask

    def materialize(self):
        self._check()
        n = _native()
        out = self.dy.new_empty(self.dy.shape)
        n._K.relu_mask_apply(self.dy.data_ptr(), self.mask.data_ptr(), out.data_ptr(),
                             self.dy.numel(), n._st())
        return out


class LazyBnDx(_Record):
    """d(x) of a residual BatchNorm + ReLU, not yet formed: dx = A (dy * mask) + B x + C per
    channel.  A fused conv backward that consumes it forms it per tile (bit-identical to the
    apply pass); anything else materialises it with that pass.  ``x`` is held strongly: it is
    the tensor whose grad slot carries this record (a cycle while the hand-off waits, broken
    when the consumer takes the record -- or by end_step)."""
    __slots__ = ("dy", "x", "mask", "gb")

    def __init__(self, dy, x, mask, gb):
        super().__init__()
        self.dy, self.x, self.mask, self.gb = dy, x, mask, gb

    def materialize(self):
        self._check()
        n = _native()
        C = self.x.shape[-1]
        M = self.x.numel() // C
        dx = self.x.new_empty(self.x.shape)
        n._materialized(self.x)
        n._K.bn_bwd_apply(self.dy.data_ptr(), 0, self.x.data_ptr(), self.gb[2].data_ptr(),
                          self.gb[3].data_ptr(), self.gb[4].data_ptr(), dx.data_ptr(), 0, M, C,
                          1, n._st(), 0, 0, self.mask.data_ptr())
        return dx


class LazyStemDz(_Record):
    """d(stem conv output) of the fused BN + ReLU + 3x3/2 max-pool (the pool's gather, the ReLU
    mask recomputed from x, dx = A dz + B x + C), not yet formed: the stem weight gradient forms
    it per strip on load (conv_wgrad_stem_dz, bit-identical to the apply pass) so it is never
    stored; anything else materialises it with that pass."""
    __slots__ = ("dp", "arg", "x", "gb", "fsc", "fsh", "geom")

    def __init__(self, dp, arg, x, gb, fsc, fsh, geom):
        super().__init__()
        self.dp, self.arg, self.x, self.gb = dp, arg, x, gb
        self.fsc, self.fsh, self.geom = fsc, fsh, geom

    def materialize(self):
        self._check()
        n = _native()
        N, H, W, C, P, Q = self.geom
        dx = self.x.new_empty(self.x.shape)
        n._K.pool_bn_bwd_apply(self.dp.data_ptr(), self.arg.data_ptr(), self.x.data_ptr(),
                               self.gb[2].data_ptr(), self.gb[3].data_ptr(),
                               self.gb[4].data_ptr(), self.fsc.data_ptr(), self.fsh.data_ptr(),
                               dx.data_ptr(), N, H, W, C, P, Q, n._st())
        return dx


class GradSlot(_Record):
    """A mailbox between two ops' backward passes: the producer's backward leaves a gradient
    record in ``grad``, the consumer's backward takes it."""
    __slots__ = ("grad",)

    def __init__(self):
        super().__init__()
        self.grad = None

    def release(self):
        g = self.grad
        super().release()
        if isinstance(g, _Record):
            g.release()


def live_count():
    """Records created since the last :func:`end_step` that are still referenced somewhere."""
    return len(_LIVE)


def end_step():
    """The training step's backward has returned: release every record still alive (their
    consumers ran or never will); returns how many were released."""
    recs = list(_LIVE)
    for r in recs:
        r.release()
    _LIVE.clear()
    return len(recs)


__all__ = ["BnDeferred", "Recompute", "MaskedGrad", "LazyBnDx", "LazyStemDz", "GradSlot",
           "ReleasedRecordError", "live_count", "end_step"]
