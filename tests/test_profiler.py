"""Step-phase timers (HIP events on GPU, perf_counter on CPU) and roctx ranges."""
import torch

import distributedtensorflow_amd as dtf
from distributedtensorflow_amd import ops
from distributedtensorflow_amd.models import MnistMLP
from distributedtensorflow_amd.optimizers import AdamOptimizer
from distributedtensorflow_amd.parallel import OneDeviceStrategy


def test_step_timer_phases_cpu():
    timer = dtf.profiler.enable("cpu")
    try:
        m = MnistMLP()
        with OneDeviceStrategy("cpu").scope():
            opt = AdamOptimizer(1e-3)
            for _ in range(3):
                with timer.phase("forward"):
                    loss = ops.sparse_softmax_cross_entropy(m(torch.rand(32, 784)),
                                                            torch.randint(0, 10, (32,)))
                opt.minimize(loss)
        s = timer.summary()
        assert set(s) == {"forward", "backward", "comm", "optimizer"}
        assert all(v >= 0 for v in s.values())
        assert timer.summary() == {}
    finally:
        dtf.profiler.disable()


def test_roctx_range_is_safe_without_library():
    with dtf.profiler.range("x"):
        pass
