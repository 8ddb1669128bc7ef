"""The deferred-work records that native ops hang on their output tensors (BN on load:
``_BnDeferred``; lazy c3 output: ``_Recompute``) must not form reference cycles with those
tensors: a cycle leaves every step's activation to Python's cyclic collector (round 5 measured
+2.9 GB of peak memory per ResNet-50 step, profiles/measurements/r5_bnl_reference_cycle_fix.jsonl).
CPU-only: the records are plain Python objects; nothing here launches a kernel."""
import gc

import torch

from distributedtensorflow_amd.ops import native


def _freed_without_collector(make_record, attr):
    was = gc.isenabled()
    gc.disable()
    try:
        out = torch.empty(64)
        rec = make_record(out)
        setattr(out, attr, rec)
        del out
        return rec.out() if hasattr(rec, "out") else rec.y()
    finally:
        if was:
            gc.enable()


def test_bn_deferred_record_does_not_keep_its_output_alive():
    x, sc, sh = torch.empty(64), torch.ones(8), torch.zeros(8)
    left = _freed_without_collector(lambda y: native._BnDeferred(x, sc, sh, y), "_dtf_bnl")
    assert left is None


def test_lazy_x3_record_does_not_keep_its_output_alive():
    y2, wb = torch.empty(8, 8), torch.empty(8, 8)
    left = _freed_without_collector(lambda out: native._Recompute(y2, wb, out), "_dtf_recompute")
    assert left is None
