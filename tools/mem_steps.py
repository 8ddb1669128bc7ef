"""Live-tensor bytes after each of a few ResNet-50 training steps with the cyclic collector off
(the check of tests/test_resnet_gpu.py::test_training_step_frees_its_activations_without_the_
cycle_collector, printed instead of asserted), and the tensors that differ between two steps'
ends -- for chasing a deferred-work record that outlives its step.

    python tools/mem_steps.py [--batch 8] [--steps 4]
"""
import argparse
import collections
import gc
import json

import torch

from distributedtensorflow_amd.models import resnet50


def live_tensors():
    out = collections.Counter()
    for o in gc.get_objects():
        try:
            if torch.is_tensor(o) and o.is_cuda:
                out[(tuple(o.shape), str(o.dtype))] += 1
        except Exception:
            pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--after", default="", help="a tests/test_resnet_gpu.py test function to run "
                    "first (the pytest order in which a leftover of that test shows)")
    a = ap.parse_args()
    if a.after:
        import os
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
        import test_resnet_gpu
        getattr(test_resnet_gpu, a.after)()
        from distributedtensorflow_amd.ops import native
        native._WT_PENDING.clear()
        native._WT_CACHE.clear()
    torch.manual_seed(0)
    m = resnet50().cuda()
    x = torch.randn(a.batch, 224, 224, 3, device="cuda").bfloat16()
    lab = torch.randint(0, 1000, (a.batch,), device="cuda")
    gc.collect()
    gc.disable()
    after, snaps = [], []
    for _ in range(a.steps):
        loss = torch.nn.functional.cross_entropy(m(x).float(), lab)
        loss.backward()
        del loss
        for p in m.parameters():
            p.grad = None
        torch.cuda.synchronize()
        after.append(torch.cuda.memory_allocated())
        snaps.append(live_tensors())
    gc.enable()
    print(json.dumps({"after": after, "spread": max(after[1:]) - min(after[1:])}))
    for i in range(1, len(snaps)):
        d = snaps[i] - snaps[i - 1]
        e = snaps[i - 1] - snaps[i]
        print(json.dumps({"step": i, "more": [[list(k[0]), k[1], v] for k, v in d.items()],
                          "fewer": [[list(k[0]), k[1], v] for k, v in e.items()]}))


if __name__ == "__main__":
    main()
