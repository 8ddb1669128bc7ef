"""ConfigProto / GPUOptions (``templates/00_mnist_replica.py:213-217``,
``run_mnist_distributed.py:122-124``): device-filter parsing and matching, the refusal of filters
that hide every parameter server, placement logging, GPU options on a CPU-only host."""
import io

import pytest
import torch

from distributedtensorflow_amd.train import session as S


def test_parse_device_filter_forms():
    assert S.parse_device_filter("/job:ps") == ("ps", None)
    assert S.parse_device_filter("/job:worker/task:3") == ("worker", 3)
    assert S.parse_device_filter("/job:worker/replica:0/task:1/device:GPU:0") == ("worker", 1)
    with pytest.raises(ValueError):
        S.parse_device_filter("/task:1")
    with pytest.raises(ValueError):
        S.parse_device_filter("/job:ps/shard:2")


def test_device_visible_reference_filter():
    # the reference template's filter for worker 1
    cfg = S.ConfigProto(device_filters=["/job:ps", "/job:worker/task:1"])
    assert cfg.device_visible("ps", 0) and cfg.device_visible("ps", 5)
    assert cfg.device_visible("worker", 1)
    assert not cfg.device_visible("worker", 0)
    assert not cfg.device_visible("chief", 0)
    assert S.ConfigProto().device_visible("worker", 7)      # no filters: everything visible


class _Cluster:
    def __init__(self, n):
        self.n = n

    def num_tasks(self, job):
        return self.n if job == "ps" else 2


class _Server:
    def __init__(self, n):
        self.cluster = _Cluster(n)


class _Strategy:
    def __init__(self, n):
        self.server = _Server(n)


def test_filters_hiding_every_ps_are_refused():
    ok = S.ConfigProto(device_filters=["/job:ps", "/job:worker/task:0"])
    ok.check_placement(_Strategy(2))
    bad = S.ConfigProto(device_filters=["/job:worker/task:0"])
    with pytest.raises(ValueError, match="hide every /job:ps"):
        bad.check_placement(_Strategy(2))
    bad.check_placement(_Strategy(0))                        # no PS tasks: nothing to hide
    part = S.ConfigProto(device_filters=["/job:ps/task:1"])
    part.check_placement(_Strategy(2))                       # one PS task visible


def test_gpu_options_from_dict_and_cpu_noop():
    cfg = S.ConfigProto(gpu_options={"per_process_gpu_memory_fraction": 0.5, "allow_growth": True})
    assert isinstance(cfg.gpu_options, S.GPUOptions)
    assert cfg.gpu_options.per_process_gpu_memory_fraction == 0.5
    if not torch.cuda.is_available():
        assert cfg.gpu_options.apply() is None
    cfg.apply()


def test_log_placement_lists_every_variable():
    from distributedtensorflow_amd.models.mnist import MnistMLP
    m = MnistMLP()
    buf = io.StringIO()
    S.log_placement(model=m, out=buf)
    lines = buf.getvalue().strip().splitlines()
    assert len(lines) == len(list(m.parameters()))
    assert lines[0].startswith("hid_w (784, 100): cpu")
