"""The N > 1 communication path on REAL RCCL, on a one-GPU box.

RCCL refuses two ranks on one device, so the driver's 8-GPU bench would be the first execution
of the bucketed all-reduce / reduce-scatter / all-gather code on RCCL.  ``DTF_FORCE_REDUCER=1``
builds the process group and the communicating reducer at world size 1: under
``torch.distributed.run --nproc-per-node 1`` on the ``nccl`` backend every backward hook, every
async collective on views of the flat gradient / master buffers (ordered against the native
ops' direct gradient writes on the compute stream), ``finish()``, the owner apply and the
overlapped variable gathers run on RCCL.  At world 1 every collective is an identity, so the
final weights must equal the plain single-process run BIT FOR BIT (the native step is
run-to-run deterministic, tools/determinism_probe.py): any bookkeeping error of the reducers --
a bucket applied twice or not at all, an owner chunk or gather range off by one, a gradient
scale, a variable read before its gather was waited for and copied into the bf16 shadow --
shows up as a difference.  (Ordering against the compute stream is by construction: every
collective is issued after the gradient writes it covers were enqueued on the current stream,
and ProcessGroupNCCL makes its stream wait on the current stream at issue.)
"""
import json
import os
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.gpu

ARGS = ["--gpus", "1", "--batch", "32", "--image-size", "128", "--steps", "3", "--warmup", "2"]


def _bench(tmp_path, name, extra, forced, comm="c10d"):
    from distributedtensorflow_amd.cluster.launcher import free_ports
    dump = tmp_path / f"{name}.pt"
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4",
               DTF_FORCE_REDUCER="1" if forced else "0", DTF_COMM=comm)
    if forced:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               "1", "--master-addr", "127.0.0.1", "--master-port", str(free_ports(1)[0]),
               os.path.join(ROOT, "bench.py")]
    else:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")]
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
    r = subprocess.run(cmd + ARGS + list(extra) + ["--dump-master", str(dump)], env=env,
                       cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), torch.load(dump, weights_only=True)


@pytest.mark.parametrize("extra,reducer,comm", [
    ((), "BucketedAllReduce", "c10d"),
    (("--strategy", "ps", "--num-ps", "1"), "_ColocatedPSReducer", "c10d"),
    (("--bucket-mb", "16"), "BucketedAllReduce", "c10d"),
    ((), "BucketedAllReduce", "rccl"),
    (("--strategy", "ps", "--num-ps", "1"), "_ColocatedPSReducer", "rccl"),
], ids=["mirrored", "ps_sharded", "mirrored_16mb", "mirrored_native_rccl", "ps_native_rccl"])
def test_forced_reducer_on_rccl_is_bit_identical(tmp_path, extra, reducer, comm):
    """``comm=rccl``: the same through the native communicator (csrc/kernels/rccl_comm.cpp)."""
    rec, master = _bench(tmp_path, "forced", extra, True, comm)
    cfg = rec["config"]
    assert cfg["comm_backend"] == "nccl", cfg
    cs = cfg["comm"]
    assert cs["forced_reducer"] is True and cs["reducer"] == reducer, cs
    assert cs["buckets"] >= 2 and cs["early_launches"] >= 3 * (cs["buckets"] - 1), cs
    assert cs["communicator"] == comm, cs
    if reducer == "_ColocatedPSReducer":
        assert cs["sharded_owners"] is True
    plain_rec, plain = _bench(tmp_path, "plain", extra, False)
    assert plain_rec["config"]["comm_backend"] is None
    assert plain_rec["config"]["comm"].get("reducer") == "_NullReducer"
    assert master.shape == plain.shape
    diff = (master != plain).sum().item()
    assert diff == 0, f"{diff} of {master.numel()} master weights differ from the plain run"


def test_forced_reducer_bucket_autotune_on_rccl(tmp_path):
    """--bucket-mb auto at world 1: every candidate re-buckets the live RCCL reducer."""
    rec, _ = _bench(tmp_path, "auto", ("--bucket-mb", "auto"), True)
    cfg = rec["config"]
    assert cfg["comm_backend"] == "nccl"
    assert sorted(int(k) for k in cfg["bucket_tune_ms"]) == [16, 32, 64, 128]
    assert cfg["comm"]["early_launches"] >= 3 * (cfg["comm"]["buckets"] - 1)
