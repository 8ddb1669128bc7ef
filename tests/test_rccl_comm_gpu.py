"""The native RCCL communicator (csrc/kernels/rccl_comm.cpp via parallel/comm.py) on a GPU:
unique id through the TCPStore, ncclCommInitRank, each collective on the comm stream ordered
against the compute stream by events (one rank: RCCL refuses two ranks on one device)."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.gpu


def test_native_rccl_collectives(tmp_path):
    from distributedtensorflow_amd.cluster.launcher import free_ports
    out = tmp_path / "rccl.json"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "1", "--master-addr", "127.0.0.1", "--master-port",
                        str(free_ports(1)[0]), os.path.join(HERE, "rccl_comm_worker.py"),
                        str(out)], env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.load(open(out))
    assert res["version"] >= 22600 and res["world"] == 1
    for k in ("all_reduce", "reduce_scatter", "all_gather", "broadcast", "reduce"):
        assert res[k] is True, (k, res)
    assert res["async_error"] == 0
