"""The deferred-work records native ops hang on their output tensors (ops/records.py: BN on load
``BnDeferred``; lazy c3 output ``Recompute``; unformed residual-BN d(x) ``LazyBnDx`` in a
``GradSlot``; masked residual gradient ``MaskedGrad``) follow one lifetime rule:

1. a record never holds a strong reference to the tensor it is attached to -- a cycle leaves every
   step's activation to Python's cyclic collector (round 5 measured +2.9 GB of peak memory per
   ResNet-50 step, profiles/measurements/r5_bnl_reference_cycle_fix.jsonl);
2. ``end_step()`` (run by ``Optimizer.compute_gradients`` after backward) releases every record
   still alive -- including a hand-off whose consumer never ran -- so none outlives its step.

CPU-only: the records are plain Python objects; nothing here launches a kernel (the GPU side:
tests/test_resnet_gpu.py::test_no_record_outlives_its_step)."""
import gc
import weakref

import pytest
import torch

from distributedtensorflow_amd.ops import records


@pytest.fixture(autouse=True)
def _no_collector():
    records.end_step()
    was = gc.isenabled()
    gc.disable()
    yield
    records.end_step()
    if was:
        gc.enable()


def _freed_without_collector(make_record, attr):
    out = torch.empty(64)
    rec = make_record(out)
    setattr(out, attr, rec)
    del out
    return rec.out() if hasattr(rec, "out") else rec.y()


def test_bn_deferred_record_does_not_keep_its_output_alive():
    x, sc, sh = torch.empty(64), torch.ones(8), torch.zeros(8)
    left = _freed_without_collector(lambda y: records.BnDeferred(x, sc, sh, y), "_dtf_bnl")
    assert left is None


def test_lazy_x3_record_does_not_keep_its_output_alive():
    y2, wb = torch.empty(8, 8), torch.empty(8, 8)
    left = _freed_without_collector(lambda out: records.Recompute(y2, wb, out), "_dtf_recompute")
    assert left is None


def test_end_step_breaks_the_waiting_lazy_dx_handoff():
    """c3's output -> its grad slot -> LazyBnDx -> that output is a cycle by construction while
    the residual BN's d(x) waits for the fused c3 backward; if that consumer never runs (a
    partial backward), end_step must still free the output."""
    out = torch.empty(1024)
    slot = records.GradSlot()
    out._dtf_lazy_slot = slot
    slot.grad = records.LazyBnDx(torch.empty(1024), out, torch.empty(128, dtype=torch.uint8),
                                 torch.empty(5, 8))
    ref = weakref.ref(out)
    del out, slot
    assert ref() is not None            # the cycle keeps it (the collector is off)
    assert records.live_count() == 2
    assert records.end_step() == 2
    assert ref() is None and records.live_count() == 0


def test_every_kind_is_released_and_refuses_late_use():
    x = torch.empty(16)
    kinds = [records.BnDeferred(x, torch.ones(2), torch.zeros(2), torch.empty(16)),
             records.Recompute(torch.empty(4, 4), torch.empty(4, 4), torch.empty(4, 4)),
             records.MaskedGrad(torch.empty(16), torch.empty(2, dtype=torch.uint8)),
             records.LazyBnDx(torch.empty(16), x, torch.empty(2, dtype=torch.uint8),
                              torch.empty(5, 2)),
             records.GradSlot()]
    held = [weakref.ref(x)]
    del x
    assert records.live_count() == len(kinds)
    records.end_step()
    assert records.live_count() == 0
    assert held[0]() is None            # LazyBnDx / BnDeferred dropped their operand
    for r in kinds:
        assert r.released
    assert kinds[0].done                # a released deferred BN is inert (nothing pending)
    for r in kinds[:4]:
        with pytest.raises(records.ReleasedRecordError):
            r.materialize()


def test_optimizer_step_releases_records():
    """compute_gradients calls ops.end_step() once backward has returned."""
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import OneDeviceStrategy
    w = torch.nn.Parameter(torch.randn(4))
    with OneDeviceStrategy("cpu").scope():
        opt = MomentumOptimizer(0.1, momentum=0.9)
        rec = records.MaskedGrad(torch.empty(4), torch.empty(1, dtype=torch.uint8))
        opt.minimize((w * w).sum(), var_list=[w])
    assert rec.released and records.live_count() == 0
