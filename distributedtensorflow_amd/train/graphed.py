"""A whole training step (forward, backward, fused optimizer update) captured once as a HIP graph
and replayed: the MI355X answer to TF1's graph executor for launch-bound steps.

TF1 builds the step as a graph and its executor walks it in C++ (``session.run(train_op)``,
reference ``run_mnist_distributed.py:113-116``).  Here the eager step runs the framework's own
HIP kernels; on a small step (the reference MNIST CNN at batch 128 is ~60 launches of a few
microseconds each) the host's per-launch cost dominates.  ``GraphedTrainStep`` records the
step's kernels on a capture stream (``torch.cuda.graph`` = hipStreamBeginCapture /
hipGraphInstantiate) and each call is one ``hipGraphLaunch``:

* every kernel of the step already launches on the caller's current stream and reads its
  per-step hyper-parameters (learning rate, Adam's lr_t, LAMB's bias corrections) from DEVICE
  buffers (``csrc/kernels/optim.hip``); the wrapper refreshes those buffers before each replay
  (``Optimizer._refresh_hyper``) and advances ``iterations`` / ``global_step`` on the host,
  exactly what the eager ``apply_gradients`` does;
* inputs live in static device buffers (``static_inputs``); ``__call__(*batch)`` copies a new
  batch in (device-to-device) before the replay;
* intermediate tensors come from the graph's private memory pool, reused by every replay.

Replays are bit-identical to eager steps (same kernels, same order; tests/test_graphed_gpu.py).
Limits: one process (no collective gradient reducer inside the graph); ops whose per-step
randomness is drawn on the host (dropout seeds) are frozen by capture, so models with dropout
are refused.
"""
from __future__ import annotations

import torch

from ..parallel.strategy import _NullReducer
from . import global_step as gs


class GraphedTrainStep:
    """``step_fn(*static_inputs)`` must run one training step (e.g. loss = model(x) ... then
    ``optimizer.minimize(loss, global_step)``) and return the tensors to read back (the loss).
    """

    def __init__(self, step_fn, optimizer, static_inputs, global_step=None, warmup=2):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedTrainStep needs a GPU (HIP graphs)")
        self.step_fn = step_fn
        self.opt = optimizer
        self.global_step = global_step
        self.static_inputs = [t if t.is_cuda else t.cuda() for t in static_inputs]
        # eager warm-up steps on a side stream: first-call initialisation (kernel attributes,
        # filter-transpose caches, optimizer build, allocator growth) must not happen in capture
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                out = step_fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if not isinstance(getattr(optimizer, "_reducer", None), _NullReducer):
            raise RuntimeError("GraphedTrainStep captures single-process steps only "
                               f"(gradient reducer {type(optimizer._reducer).__name__})")
        # capture: the host-side bookkeeping of the recorded step is rolled back (capture records
        # kernels, it does not execute them)
        it0 = optimizer.iterations
        step0 = gs_value(global_step)
        draws0 = _seed_draws()
        self.graph = torch.cuda.CUDAGraph()
        optimizer._capturing = True
        try:
            # captured on the warm-up stream: the parameters' AccumulateGrad nodes were created
            # there, and a capture on another stream makes autograd warn that the node's stream
            # does not match
            with torch.cuda.graph(self.graph, stream=side):
                self.static_out = step_fn(*self.static_inputs)
        finally:
            optimizer._capturing = False
        if _seed_draws() != draws0:
            raise RuntimeError("GraphedTrainStep: the step draws dropout seeds on the host; a "
                               "captured graph would replay one mask forever")
        optimizer.iterations = it0
        if global_step is not None:
            global_step.assign(step0)
        self.replays = 0

    def __call__(self, *inputs):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not dst:
                dst.copy_(src, non_blocking=True)
        opt = self.opt
        opt.iterations += 1                  # what apply_gradients does before the update
        opt._refresh_hyper()
        if self.global_step is not None:
            gs.increment(self.global_step)
        self.graph.replay()
        self.replays += 1
        return self.static_out


def _seed_draws():
    try:
        from ..ops import native_nlp
    except ImportError:        # no extension: no native dropout either
        return 0
    return native_nlp.SEED_DRAWS[0]


def gs_value(step):
    if step is None:
        return 0
    return int(step.value()) if hasattr(step, "value") else int(step)
