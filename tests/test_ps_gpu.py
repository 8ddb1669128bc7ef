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


def _failure_report(codes, text):
    """Exit codes, then per task its FIRST traceback (the primary failure: a later one may only
    be a consequence) and its log tail -- also printed, since pytest truncates long messages."""
    parts = [f"exit codes: {codes}"]
    for k, t in text.items():
        i = t.find("Traceback")
        first = t[i:i + 3000] if i >= 0 else "(no traceback)"
        parts.append(f"===== {k}: first traceback =====\n{first}\n===== {k}: tail =====\n"
                     f"{t[-2000:]}")
    rep = "\n".join(parts)
    print(rep)
    return rep


@pytest.mark.parametrize("pipeline", ["0", "1"], ids=["serial", "pipelined"])
def test_ps_killed_on_gpu_restarts_and_resumes(tmp_path, pipeline):
    """The recovery path on the HBM data plane: the PS dies holding its exported HBM shard,
    the launcher restarts it, the workers drop their hipIpc mappings, join generation 1 and the
    chief re-seeds the new shard from the latest checkpoint -- with the serial and with the
    pipelined push/pull (whose push in flight is cancelled and joined before leaving the old
    generation).  Every recovery wait is bounded below the job budget (DTF_RECOVERY_TIMEOUT_S,
    DTF_PS_TIMEOUT_S), so a stall names itself in a task log instead of outlasting the launcher,
    and a launcher timeout raises with every task's log tail and stacks in its message."""
    from distributedtensorflow_amd.cluster.launcher import launch_local
    ckpt = tmp_path / "ckpt"
    codes, logs = launch_local(os.path.join(ROOT, "run_mnist_distributed.py"), 1, 2,
                               str(tmp_path),
                               ["--max_steps=60", f"--data_dir={tmp_path}/data",
                                f"--log_dir={tmp_path}/tb", "--ps_device=gpu",
                                f"--checkpoint_dir={ckpt}", "--save_checkpoint_steps=10"],
                               env={"PYTHONPATH": ROOT, "DTF_FAULT_KILL_PS_AT_STEP": "30",
                                    "DTF_PS_PIPELINE": pipeline,
                                    "DTF_RECOVERY_TIMEOUT_S": "45", "DTF_PS_TIMEOUT_S": "45"},
                               timeout_s=150, grace_s=20, max_ps_restarts=1)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), _failure_report(codes, text)
    assert "restarting (1/1)" in text["ps0"]
    assert all("recovered: generation 1" in text[w] for w in ("worker0", "worker1"))
    m = re.search(r"Close Parameter Server \.\.\. (\{.*\})", text["ps0"])
    stats = ast.literal_eval(m.group(1))
    assert stats["data_plane"] == "ipc" and stats["global_step"] >= 60   # the restarted PS


def test_ps_async_bench_four_workers_concurrent_applies(tmp_path):
    """1 PS + 4 workers on the GPU data plane, pipelined push/pull (bucket
    pushes from the backward hooks, post/answer on a comm thread, per-bucket pull fences).  The
    owner runs applies of different workers concurrently on their own streams (Hogwild,
    ps_max_inflight_applies >= 2), applies every push (no drops) and the final global step
    counts every push of every worker."""
    import json
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--strategy", "ps_async",
                        "--num-workers", "4", "--batch", "8", "--image-size", "64", "--steps",
                        "8", "--warmup", "2", "--timeout", "150"],
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2"),
                       capture_output=True, text=True, timeout=200, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = rec["config"]
    assert cfg["data_plane"] == "ipc" and cfg["pipelined_push_pull"] is True
    assert cfg["ps_applied"] == cfg["ps_pushes"] == 4 * (8 + 2)
    assert cfg["final_global_step"] == 4 * (8 + 2)
    assert cfg["ps_max_inflight_applies"] >= 2, cfg
    assert rec["value"] > 0


@pytest.mark.parametrize("pipeline", ["0", "1"])
def test_pipelined_push_pull_matches_serial_one_worker(tmp_path, pipeline):
    """With ONE async worker the run is deterministic: the pipelined data plane must train
    exactly like the serial one (same pushes, same pulls, same order) -- final variables equal
    bit for bit to the serial run's."""
    from distributedtensorflow_amd.cluster.launcher import launch_local
    from distributedtensorflow_amd.train.checkpoint import latest_checkpoint, load_variable
    outs = {}
    for mode in ("0", pipeline):
        d = tmp_path / f"p{mode}_{len(outs)}"
        codes, logs = launch_local(os.path.join(ROOT, "run_mnist_distributed.py"), 1, 1, str(d),
                                   ["--max_steps=40", f"--data_dir={tmp_path}/data",
                                    f"--log_dir={d}/tb", "--ps_device=gpu", "--seed=7",
                                    f"--checkpoint_dir={d}/ckpt", "--save_checkpoint_steps=1000"],
                                   env={"PYTHONPATH": ROOT, "DTF_PS_PIPELINE": mode},
                                   timeout_s=100, grace_s=20)
        text = {k: open(v).read() for k, v in logs.items()}
        assert all(c == 0 for c in codes.values()), {k: t[-2500:] for k, t in text.items()}
        last = latest_checkpoint(str(d / "ckpt"))
        outs[len(outs)] = {n: load_variable(last, n) for n in
                           ("conv2d/kernel", "conv2d_1/kernel", "dense/kernel", "dense_1/bias",
                            "global_step")}
    a, b = outs[0], outs[1]
    assert int(a["global_step"]) == int(b["global_step"]) >= 40
    for k in a:
        assert (a[k] == b[k]).all(), k
