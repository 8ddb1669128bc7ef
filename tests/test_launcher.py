"""Launcher failure reporting: a stalled job fails at its deadline with
every task's log tail and the stalled task's stack in the exception message, and a task that
fails for good ends the job at once (the survivors are stopped, their stacks dumped) instead of
leaving them to wait out their own timeouts."""
import os
import time

import pytest

from distributedtensorflow_amd.cluster import rendezvous
from distributedtensorflow_amd.cluster.launcher import LaunchTimeout, launch_local

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
TASK = os.path.join(HERE, "launcher_task.py")


def test_stalled_task_times_out_with_logs_and_stacks(tmp_path):
    t0 = time.time()
    with pytest.raises(LaunchTimeout) as ei:
        launch_local(TASK, 1, 2, str(tmp_path), env={"LAUNCHER_TASK_MODE": "hang"},
                     timeout_s=6, grace_s=2)
    assert time.time() - t0 < 30
    msg = str(ei.value)
    assert "worker1" in ei.value.alive
    assert "===== worker1 (log tail) =====" in msg and "task worker:1 mode hang" in msg
    # the SIGUSR1 stack dump of the stalled task names the frame it was stuck in
    assert "stalled_wait" in msg


def test_task_failing_for_good_ends_the_job_at_once(tmp_path):
    t0 = time.time()
    codes, logs = launch_local(TASK, 1, 2, str(tmp_path), env={"LAUNCHER_TASK_MODE": "ps_fail",
                                                                "LAUNCHER_TASK_DIR": str(tmp_path)},
                               timeout_s=120, grace_s=2)
    assert time.time() - t0 < 40, "the workers must be stopped, not waited for"
    assert codes[("ps", 0)] == 3 and codes[("worker", 0)] != 0 and codes[("worker", 1)] != 0
    text = {k: open(v).read() for k, v in logs.items()}
    assert "is not restarted" in text["ps0"]
    assert "ps0 failed for good (exit 3); stopping worker0" in text["worker0"]
    assert "stalled_wait" in text["worker1"]          # stack dumped before the stop


@pytest.mark.parametrize("sync", [False, True])
def test_worker_failing_in_async_job_leaves_the_chief_training(tmp_path, sync):
    """in asynchronous between-graph training a worker that fails for good does not
    end the job -- the chief trains on and finishes (TF1 semantics); a synchronous job (every step
    needs every worker) is stopped at once instead."""
    codes, logs = launch_local(TASK, 1, 2, str(tmp_path),
                               env={"LAUNCHER_TASK_MODE": "worker_fail",
                                    "LAUNCHER_TASK_DIR": str(tmp_path)},
                               timeout_s=60, grace_s=5, sync=sync)
    text = {k: open(v).read() for k, v in logs.items()}
    assert codes[("worker", 1)] == 5
    if sync:
        assert codes[("worker", 0)] != 0
        assert "worker1 failed for good (exit 5); stopping worker0" in text["worker0"]
    else:
        assert codes[("worker", 0)] == 0 and codes[("ps", 0)] == 0
        assert "the other tasks continue" in text["worker1"]
        assert "stopping" not in text["worker0"] and "stopping" not in text["ps0"]


def test_epoch_arrival_barrier_names_the_missing_rank():
    import datetime

    import torch.distributed as dist
    from distributedtensorflow_amd.cluster.launcher import free_ports
    port = free_ports(1)[0]
    store = dist.TCPStore("127.0.0.1", port, None, True, timeout=datetime.timedelta(seconds=10),
                          wait_for_workers=False)
    t0 = time.time()
    with pytest.raises(TimeoutError, match=r"rank\(s\) \[1, 2\] of 3 to join cluster epoch 4"):
        rendezvous.arrive(store, 4, 0, 3, 0.5, "worker:0")
    assert time.time() - t0 < 3


def test_recovery_timeout_env(monkeypatch):
    monkeypatch.delenv("DTF_RECOVERY_TIMEOUT_S", raising=False)
    assert rendezvous.recovery_timeout_s() == 120.0
    monkeypatch.setenv("DTF_RECOVERY_TIMEOUT_S", "7")
    assert rendezvous.recovery_timeout_s() == 7.0


def test_process_group_timeout_exceeds_watchdog_deadline():
    """c10d's own timeout must never fire before the DTF watchdog's deadline."""
    from distributedtensorflow_amd.parallel.strategy import pg_timeout_for
    for d in (1, 30, 300, 1800):
        assert pg_timeout_for(d) > d and pg_timeout_for(d) >= 2 * d
