"""Restart-from-checkpoint of a collective world on the GPU's RCCL path (VERDICT r3, next-round
item 2; reference: MonitoredTrainingSession recreating the session after a preempted task,
/root/reference/run_mnist_distributed.py:128-132,146).

One rank under ``launch_collective`` on the ``nccl`` backend with the communicating reducer forced
on (``DTF_FORCE_REDUCER=1``: the process group, the bucket hooks and every collective of the
N > 1 path run), over both communicators (c10d ProcessGroupNCCL and the native ``ncclComm_t``).
The rank is SIGKILLed at global step 5 in its first life; the launcher restarts it in a new
cluster epoch, the new process restores the latest checkpoint (step 3), re-creates the RCCL
communicator under the new epoch's store keys and trains to step 12.  Its final fp32 masters must
equal, bit for bit, those of an uninterrupted run -- i.e. the restore is exact and the resumed
steps are the same steps.

(Survivors released from a blocked RCCL kernel need >= 2 GPUs: that part is covered by the
watchdog unit tests and the 2-rank gloo hung-peer test in tests/test_watchdog.py.)"""
import os

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.gpu


def _run(tmp, comm, fault):
    from distributedtensorflow_amd.cluster.launcher import launch_collective
    env = {"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2", "DTF_FORCE_REDUCER": "1",
           "DTF_COMM": comm, "DTF_COMM_TIMEOUT_S": "60"}
    if fault:
        env["DTF_FAULT_SIGKILL"] = "rank:0@5"
    codes, logs = launch_collective(os.path.join(HERE, "dist_worker.py"), 1, str(tmp),
                                    ["mirrored_recovery", str(tmp), "steps=12", "save=3",
                                     "strategy=mirrored", "opt=adam"],
                                    env=env, timeout_s=100, max_restarts=1 if fault else 0)
    text = open(logs["rank0"]).read()
    assert codes[0] == 0, text[-4000:]
    return torch.load(tmp / "rank0.pt", weights_only=True), text


@pytest.mark.parametrize("comm", ["c10d", "rccl"])
def test_killed_rank_restarts_from_checkpoint_on_nccl(tmp_path, comm):
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    killed, text = _run(tmp_path / "a", comm, fault=True)
    assert "fault injection: SIGKILL rank:0" in text
    assert "restarting (1/1), cluster epoch 1" in text, text[-3000:]
    assert killed["restart"] == 1 and killed["global_step"] == 12
    assert killed["comm"] == comm and killed["reducer"] == "BucketedAllReduce"
    clean, _ = _run(tmp_path / "b", comm, fault=False)
    assert clean["restart"] == 0 and clean["global_step"] == 12
    assert torch.equal(killed["master"], clean["master"])
    for k in clean["state"]:
        assert torch.equal(killed["state"][k], clean["state"][k]), k
