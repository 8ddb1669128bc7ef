"""Rehearsal of the driver's multi-GPU bench launch on a one-GPU box.

The round-end driver runs ``bench.py --gpus N`` under ``torch.distributed.run`` with one rank per
GPU over RCCL.  RCCL refuses two ranks on one device, so here two ``bench.py`` ranks share
cuda:0 over gloo (``DTF_BENCH_BACKEND=gloo``).  Everything else is the N > 1 path of the bench:
the bucketed all-reduce hooks firing during backward, the exposed-comm figures, the MAX-over-ranks
timing and the rank-0 JSON line.  Both the mirrored strategy and the colocated parameter-server
strategy (BASELINE config 4) run.
"""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.gpu


def _run_two_ranks(tmp_path, extra):
    from distributedtensorflow_amd.cluster.launcher import free_ports
    port = free_ports(1)[0]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT,
                   OMP_NUM_THREADS="2", DTF_BENCH_BACKEND="gloo")
        out = open(tmp_path / f"rank{r}.out", "w")
        err = open(tmp_path / f"rank{r}.err", "w")
        procs.append((subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "16",
             "--image-size", "96", "--steps", "3", "--warmup", "2", *extra],
            env=env, stdout=out, stderr=err, cwd=ROOT), out, err))
    try:
        for p, _, _ in procs:
            p.wait(timeout=100)
    finally:
        for p, out, err in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
            out.close()
            err.close()
    for r, (p, _, _) in enumerate(procs):
        assert p.returncode == 0, open(tmp_path / f"rank{r}.err").read()[-3000:]
    lines = [ln for ln in open(tmp_path / "rank0.out").read().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, lines
    # only rank 0 reports (gloo itself may print a connection line)
    assert not any(ln.startswith("{") for ln in open(tmp_path / "rank1.out").read().splitlines())
    return json.loads(lines[0])


def test_bench_two_ranks_mirrored(tmp_path):
    rec = _run_two_ranks(tmp_path, [])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 2
    cfg = rec["config"]
    assert cfg["global_batch"] == 32 and cfg["per_gpu_batch"] == 16
    assert cfg["parallelism"] == "dp2"
    assert cfg["comm_backend"] == "gloo" and cfg["backend"] != "reference"
    assert cfg["native_ext"].startswith("distributedtensorflow_amd/_lib/_dtf_hip")
    comm = cfg["comm"]
    assert comm["buckets"] >= 2 and comm["steps"] == 3
    # every bucket but the last launches from a backward hook, before backward returns
    assert comm["early_launches"] >= 3 * (comm["buckets"] - 1), comm
    assert comm["exposed_ms_per_step"] >= 0.0
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    assert abs(rec["value"] - 32 * 1000.0 / rec["ms_per_step"]) / rec["value"] < 1e-3
    assert rec["config"]["final_loss"] == rec["config"]["final_loss"]   # finite, not NaN


def test_bench_two_ranks_colocated_ps(tmp_path):
    rec = _run_two_ranks(tmp_path, ["--strategy", "ps", "--num-ps", "1"])
    cfg = rec["config"]
    assert cfg["parallelism"] == "ps1+dp2"
    assert cfg["comm_backend"] == "gloo"
    # the owner reduces and broadcasts on the same bucket plan, launched from backward hooks
    assert cfg["comm"]["buckets"] >= 2 and cfg["comm"]["early_launches"] >= 3
    assert rec["value"] > 0


def test_bench_two_ranks_sharded_ps(tmp_path):
    """num_ps == world: reduce-scatter push / owner apply / overlapped all-gather pull."""
    rec = _run_two_ranks(tmp_path, ["--strategy", "ps", "--num-ps", "2"])
    cfg = rec["config"]
    assert cfg["parallelism"] == "ps2+dp2"
    assert cfg["comm"]["sharded_owners"] is True
    assert cfg["comm"]["buckets"] >= 2 and cfg["comm"]["early_launches"] >= 3
    assert rec["value"] > 0 and cfg["final_loss"] == cfg["final_loss"]


def test_bench_two_ranks_bucket_autotune(tmp_path):
    """--bucket-mb auto: every candidate re-buckets the live reducer (hooks detached and
    re-registered), the rank-max timing picks one, and the timed steps run on it."""
    rec = _run_two_ranks(tmp_path, ["--bucket-mb", "auto"])
    cfg = rec["config"]
    tune = cfg["bucket_tune_ms"]
    assert sorted(int(k) for k in tune) == [16, 32, 64, 128]
    assert all(v > 0 for v in tune.values())
    best = min(tune, key=tune.get)
    assert cfg["bucket_mb"] == float(best)
    comm = cfg["comm"]
    assert comm["steps"] == 3 and comm["early_launches"] >= 3 * (comm["buckets"] - 1)


def test_bench_two_ranks_bert(tmp_path):
    """BASELINE config 5 flow at N = 2: BERT-base MLM under MultiWorkerMirroredStrategy (fused
    LAMB, bucketed all-reduce), tokens/sec JSON from rank 0."""
    rec = _run_two_ranks(tmp_path, ["--model", "bert_base", "--seq-len", "64",
                                    "--max-predictions", "10"])
    cfg = rec["config"]
    assert rec["unit"] == "tokens/sec" and cfg["model"] == "bert_base"
    assert cfg["parallelism"] == "dp2" and cfg["global_batch"] == 32
    assert cfg["comm_backend"] == "gloo" and cfg["comm"]["buckets"] >= 2
    assert cfg["comm"]["early_launches"] >= 3
    assert abs(rec["value"] - 32 * 64 * 1000.0 / rec["ms_per_step"]) / rec["value"] < 1e-3


def test_bench_self_launches_n_ranks_without_torchrun(tmp_path):
    """a plain ``python bench.py --gpus 2`` (no torchrun env) starts the two
    rank processes itself -- here sharing cuda:0 over gloo, the one-GPU rehearsal -- and rank 0
    reports the whole 2-rank job."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT")}
    env.update(PYTHONPATH=ROOT, OMP_NUM_THREADS="2", DTF_BENCH_BACKEND="gloo",
               DTF_BENCH_SHARE_DEVICE="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--batch", "16", "--image-size", "96", "--steps", "3", "--warmup", "2"],
                       env=env, capture_output=True, text=True, timeout=150, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    rec = json.loads(lines[0])
    cfg = rec["config"]
    assert rec["n_gpus"] == 2 and cfg["parallelism"] == "dp2" and cfg["global_batch"] == 32
    assert cfg["comm"]["buckets"] >= 2
    assert cfg["launch"]["mode"] == "self"
    assert cfg["launch"]["env_world_size"] == 2 and cfg["launch"]["dist_world_size"] == 2


def test_bench_nccl_refuses_more_ranks_than_gpus():
    """--gpus N on RCCL with fewer visible GPUs exits non-zero fast with the device-count reason
    (never a silent 1-GPU number labelled N, never a hang)."""
    import time
    import torch
    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "DTF_BENCH_BACKEND",
                        "DTF_BENCH_SHARE_DEVICE")}
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--steps", "1", "--warmup", "1"], env=env, capture_output=True,
                       text=True, timeout=60, cwd=ROOT)
    assert p.returncode != 0
    assert "refusing to measure fewer GPUs" in p.stderr, p.stderr[-2000:]
    assert time.time() - t0 < 30


def _run_ranks(tmp_path, n, extra, timeout=150):
    from distributedtensorflow_amd.cluster.launcher import free_ports
    port = free_ports(1)[0]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK="0",
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   PYTHONPATH=ROOT, OMP_NUM_THREADS="2", DTF_BENCH_BACKEND="gloo")
        out = open(tmp_path / f"rank{r}.out", "w")
        err = open(tmp_path / f"rank{r}.err", "w")
        procs.append((subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--batch", "8",
             "--image-size", "64", "--steps", "3", "--warmup", "2", *extra],
            env=env, stdout=out, stderr=err, cwd=ROOT), out, err))
    try:
        for p, _, _ in procs:
            p.wait(timeout=timeout)
    finally:
        for p, out, err in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
            out.close()
            err.close()
    return [p.returncode for p, _, _ in procs]


@pytest.mark.parametrize("strategy", ["mirrored", "ps"])
def test_bench_four_ranks_reports_per_rank_diagnostics(tmp_path, strategy):
    """the N > 1 JSON carries what a first 1 -> 8 scaling run needs to be
    read -- per-rank step time (min / max / each rank), every rank's bucket count, bucket-plan and
    collective issue-order hashes (identical, or the run fails), exposed comm time per rank and
    the RCCL channel count (None on this gloo rehearsal: 4 ranks sharing cuda:0)."""
    extra = [] if strategy == "mirrored" else ["--strategy", "ps", "--num-ps", "4"]
    codes = _run_ranks(tmp_path, 4, extra)
    assert codes == [0] * 4, open(tmp_path / "rank0.err").read()[-3000:]
    lines = [ln for ln in open(tmp_path / "rank0.out").read().splitlines() if ln.startswith("{")]
    rec = json.loads(lines[-1])
    ranks = rec["config"]["comm"]["ranks"]
    assert rec["n_gpus"] == 4 and len(ranks["ms_per_step"]) == 4
    assert ranks["ms_per_step_min"] <= ranks["ms_per_step_max"]
    # the reported step time is the slowest rank's (MAX over ranks)
    assert abs(rec["ms_per_step"] - ranks["ms_per_step_max"]) <= 0.01 * rec["ms_per_step"] + 0.01
    assert len(set(ranks["buckets"])) == 1 and ranks["buckets"][0] >= 2
    assert len(set(ranks["plan_hash"])) == 1 and len(set(ranks["order_hash"])) == 1
    assert sorted(ranks["issue_order_rank0"]) == list(range(ranks["buckets"][0]))
    assert len(ranks["exposed_comm_ms_per_step"]) == 4
    assert ranks["rccl_channels"] == [None] * 4


def test_bench_rank_with_another_bucket_order_fails(tmp_path):
    """A rank issuing its bucket collectives in another order makes the bench exit non-zero
    (order check or comm deadline), never report a number."""
    os.environ["DTF_DEBUG_PERTURB_BUCKET_ORDER"] = "1"
    os.environ["DTF_COMM_TIMEOUT_S"] = "10"
    try:
        codes = _run_ranks(tmp_path, 2, [], timeout=120)
    finally:
        del os.environ["DTF_DEBUG_PERTURB_BUCKET_ORDER"], os.environ["DTF_COMM_TIMEOUT_S"]
    assert any(c != 0 for c in codes)
    out = open(tmp_path / "rank0.out").read()
    assert not any(ln.startswith("{") for ln in out.splitlines())
