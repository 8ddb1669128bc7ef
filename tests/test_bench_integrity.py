"""bench.py integrity: the configuration a bench line claims is the one it ran.

* ``--strategy ps_async`` honours ``--gpus N``: one worker per GPU (cuda:0 .. N-1), the PS task
  colocated on cuda:0, ``n_gpus`` = the devices actually used, and a refusal when fewer GPUs are
  visible than requested;
* wrong-result timing probes cannot be benchmarked (env vars refused, probe builds refused);
* every ``DTF_*`` variable is recorded in the JSON (``config.dtf_env``);
* at N > 1 the all-reduce bucket size is auto-tuned by default.
"""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _bench(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env.update(PYTHONPATH=ROOT, **(env_extra or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=ROOT)


def test_ps_async_device_plan():
    from distributedtensorflow_amd.utils.ps_bench import device_plan
    # BASELINE config 4 on a node: 8 workers on cuda:0..7, the PS colocated on cuda:0
    assert device_plan(8, 8, 8) == (list(range(8)), 0)
    # more workers than GPUs share them round-robin; fewer GPUs requested than visible: only N
    assert device_plan(4, 2, 8) == ([0, 1, 0, 1], 0)
    assert device_plan(1, 1, 1) == ([0], 0)
    # a CPU-only host runs the flow with no devices at N = 1
    assert device_plan(2, 1, 0) == ([None, None], None)
    with pytest.raises(ValueError, match="refusing to measure fewer GPUs"):
        device_plan(4, 4, 1)
    with pytest.raises(ValueError, match="refusing to measure fewer GPUs"):
        device_plan(8, 8, 0)


def test_ps_async_refuses_more_gpus_than_visible():
    import torch
    n = torch.cuda.device_count() + 3
    r = _bench(["--strategy", "ps_async", "--gpus", str(n), "--steps", "1", "--warmup", "1"])
    assert r.returncode != 0
    assert "refusing to measure fewer GPUs" in r.stderr, r.stderr[-2000:]


@pytest.mark.parametrize("var", ["DTF_BNL_PROBE", "DTF_STREAM_BNB_PROBE", "DTF_ANY_PROBE_X"])
def test_bench_refuses_timing_probe_env(var):
    r = _bench(["--steps", "1", "--warmup", "1"], {var: "1"})
    assert r.returncode != 0
    assert "timing-probe variables set" in r.stderr and var in r.stderr, r.stderr[-2000:]
    r = _bench(["--strategy", "ps_async", "--steps", "1", "--warmup", "1"], {var: "1"})
    assert r.returncode != 0 and "timing-probe" in r.stderr


def test_smoke_refuses_timing_probe_env():
    env = dict(os.environ, PYTHONPATH=ROOT, DTF_BNL_PROBE="1")
    r = subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.smoke()"], env=env,
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode != 0 and "timing-probe" in r.stderr + r.stdout


def test_default_build_has_no_probes():
    """The wrong-result probes are compiled only into a -DDTF_PROBES build; the default build
    refuses to switch them on."""
    pytest.importorskip("distributedtensorflow_amd._lib._dtf_hip")
    from distributedtensorflow_amd._lib import _dtf_hip as K
    assert K.probes_built() is False
    with pytest.raises(RuntimeError, match="DTF_PROBES"):
        K.conv_set_bnl_probe(1)
    with pytest.raises(RuntimeError, match="DTF_PROBES"):
        K.gemm_stream_set_bnb_probe(4)
    K.conv_set_bnl_probe(0)            # switching off is always allowed
    assert not any("PROBE" in line and "os.environ" in line
                   for line in open(os.path.join(ROOT, "distributedtensorflow_amd", "ops",
                                                 "native.py")))


def test_dtf_env_recorded(monkeypatch):
    from distributedtensorflow_amd.utils import dtf_env
    for k in list(os.environ):
        if k.startswith("DTF_"):
            monkeypatch.delenv(k)
    assert dtf_env() == {}
    monkeypatch.setenv("DTF_GEMM_STREAM", "0")
    monkeypatch.setenv("DTF_BENCH_LAUNCH", "self")       # plumbing, not configuration
    assert dtf_env() == {"DTF_GEMM_STREAM": "0"}


def test_bucket_size_auto_by_default_at_n_gt_1(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    a = bench.parse()
    assert a.bucket_auto and a.num_workers == 8
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert not a.bucket_auto and a.bucket_mb == 64.0 and a.num_workers == 1
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--bucket-mb", "32"])
    a = bench.parse()
    assert not a.bucket_auto and a.bucket_mb == 32.0
