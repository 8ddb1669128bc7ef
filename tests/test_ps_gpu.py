"""Between-graph parameter server on the GPU data plane (HBM shard + hipIpc mappings).

The reference's own mode (``run_mnist_distributed.py``: 1 PS + N workers, async Adam; the
SyncReplicas template) with every task a process on the MI355X: the PS keeps its shard in HBM,
workers write gradients into their mailbox slots and read variables back through hipIpc
mappings of the owner's buffers (parallel/ps_device.py)."""
import ast
import os
import re

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, num_workers, steps, *flags):
    from distributedtensorflow_amd.cluster.launcher import launch_local
    codes, logs = launch_local(os.path.join(ROOT, "run_mnist_distributed.py"), 1, num_workers,
                               str(tmp_path),
                               [f"--max_steps={steps}", f"--data_dir={tmp_path}/data",
                                f"--log_dir={tmp_path}/tb", "--ps_device=gpu", *flags],
                               env={"PYTHONPATH": ROOT}, timeout_s=100, grace_s=20)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-2500:] for k, t in text.items()}
    m = re.search(r"Close Parameter Server \.\.\. (\{.*\})", text["ps0"])
    assert m, text["ps0"][-2000:]
    return text, ast.literal_eval(m.group(1))


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def test_async_ps_hbm_shard_ipc(tmp_path):
    text, stats = _run(tmp_path, 2, 120)
    assert stats["data_plane"] == "ipc"
    assert stats["applied"] == stats["pushes"] >= 120       # apply on arrival, nothing dropped
    lines = re.findall(r"loss = ([0-9.]+) \(global step: (\d+)\)", text["worker0"])
    steps = [int(s) for _, s in lines]
    assert steps == sorted(steps) and steps[-1] >= 120
    assert float(lines[-1][0]) < float(lines[0][0])


def test_sync_replicas_ps_hbm_shard_ipc(tmp_path):
    text, stats = _run(tmp_path, 2, 30, "--sync_replicas")
    assert stats["data_plane"] == "ipc"
    steps = [int(s) for s in re.findall(r"global step: (\d+)\)", text["worker0"])]
    assert len(set(steps)) == len(steps) and steps[-1] >= 30
    # every push was either summed into a step or dropped (stale / backup), never lost; every
    # applied step consumed at most replicas_to_aggregate = 2 gradients, and all but the last
    # (closed early when the other worker stopped) exactly 2
    assert stats["pushes"] == stats["aggregated"] + stats["dropped_stale"]
    assert 2 * stats["applied"] - 1 <= stats["aggregated"] <= 2 * stats["applied"]
    assert stats["applied"] == stats["global_step"] >= 30


def test_ps_killed_on_gpu_restarts_and_resumes(tmp_path):
    """The recovery path on the HBM data plane: the PS dies holding its exported HBM shard,
    the launcher restarts it, the workers drop their hipIpc mappings, join generation 1 and the
    chief re-seeds the new shard from the latest checkpoint."""
    from distributedtensorflow_amd.cluster.launcher import launch_local
    ckpt = tmp_path / "ckpt"
    codes, logs = launch_local(os.path.join(ROOT, "run_mnist_distributed.py"), 1, 2,
                               str(tmp_path),
                               ["--max_steps=60", f"--data_dir={tmp_path}/data",
                                f"--log_dir={tmp_path}/tb", "--ps_device=gpu",
                                f"--checkpoint_dir={ckpt}", "--save_checkpoint_steps=10"],
                               env={"PYTHONPATH": ROOT, "DTF_FAULT_KILL_PS_AT_STEP": "30"},
                               timeout_s=150, grace_s=20, max_ps_restarts=1)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-2500:] for k, t in text.items()}
    assert "restarting (1/1)" in text["ps0"]
    assert all("recovered: generation 1" in text[w] for w in ("worker0", "worker1"))
    m = re.search(r"Close Parameter Server \.\.\. (\{.*\})", text["ps0"])
    stats = ast.literal_eval(m.group(1))
    assert stats["data_plane"] == "ipc" and stats["global_step"] >= 60   # the restarted PS
