"""Multi-process data parallelism on CPU (gloo), the way the driver runs it on GPUs (one process
per rank, torchrun env).  SURVEY.md §4: replicas must stay bit-identical and match a
single-process run on the concatenated batch; parameter-server clusters (reference
``run_mnist_distributed.py``: 1 PS + 2 workers, async and SyncReplicas) must train and exit."""
import json
import os
import re
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import dist_worker  # noqa: E402

from distributedtensorflow_amd.cluster.launcher import free_ports, launch_local  # noqa: E402


def _launch(kind, world, tmp_path, *args, extra_env=None, timeout=240):
    port = free_ports(1)[0]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2",
                   PYTHONPATH=ROOT)
        env.update(extra_env(r) if extra_env else {})
        if extra_env:
            for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
                if k in extra_env(r) and extra_env(r)[k] is None:
                    env.pop(k)
            env = {k: v for k, v in env.items() if v is not None}
        log = open(tmp_path / f"{kind}{r}.log", "w")
        procs.append((subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"),
                                        kind, str(tmp_path), *args], env=env, stdout=log,
                                       stderr=subprocess.STDOUT), log))
    try:
        for p, _ in procs:
            p.wait(timeout=timeout)
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
            log.close()
    for r, (p, _) in enumerate(procs):
        assert p.returncode == 0, open(tmp_path / f"{kind}{r}.log").read()[-3000:]
    return [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]


def _single_process(opt="momentum", steps=3, with_opt=False):
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import MnistCNN
    from distributedtensorflow_amd.parallel import OneDeviceStrategy
    from distributedtensorflow_amd.train import global_step as gs_mod
    gs_mod.reset_global_step()
    torch.manual_seed(17)
    strat = OneDeviceStrategy("cpu")
    with strat.scope():
        model = MnistCNN()
        o = dist_worker.make_optimizer(opt)
        o.build(list(model.parameters()))
        for step in range(steps):
            x, y = dist_worker.global_batch(step)
            o.minimize(ops.sparse_softmax_cross_entropy(model(x), y))
    state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    return (state, o) if with_opt else state


def _assert_replicas(results, ref, atol=2e-6, steps=3):
    assert all(r["fingerprints"] == results[0]["fingerprints"] for r in results)
    for r in results[1:]:
        for k in ref:
            assert torch.equal(r["state"][k], results[0]["state"][k]), f"replicas diverged at {k}"
    for k in ref:
        torch.testing.assert_close(results[0]["state"][k], ref[k], atol=atol, rtol=1e-5)
    assert all(r["global_step"] == steps for r in results)


@pytest.mark.parametrize("args", [(), ("bucket_mb=0.05",), ("bucket_mb=0.05", "direct=1")],
                         ids=["default_buckets", "many_buckets", "direct_grad_writes"])
def test_mirrored_two_ranks_matches_single_process(tmp_path, args):
    res = _launch("mirrored", 2, tmp_path, *args)
    _assert_replicas(res, _single_process())
    assert res[0]["mean_loss"] == res[1]["mean_loss"]


@pytest.mark.parametrize("kind,args", [("mirrored", ("bucket_mb=0.05",)),
                                       ("colocated_ps", ("bucket_mb=0.05", "num_ps=2",
                                                         "opt=adam"))],
                         ids=["mirrored", "colocated_ps"])
def test_buckets_launch_during_backward(tmp_path, kind, args):
    """Overlap: every bucket but (at most) the last is launched from the post-accumulate hooks,
    i.e. before loss.backward() returned -- the negative control (hooks off) launches none."""
    res = _launch(kind, 2, tmp_path, *args)
    for r in res:
        assert r["early_launches"], "no bucket statistics recorded"
        for early, n in r["early_launches"]:
            assert n >= 3 and early >= n - 1, r["early_launches"]
    off = _launch("mirrored", 2, tmp_path, "bucket_mb=0.05", "overlap=0")
    _assert_replicas(off, _single_process())
    assert all(e == 0 for r in off for e, _ in r["early_launches"])


def test_mirrored_bf16_gradient_compression(tmp_path):
    res = _launch("mirrored", 2, tmp_path, "bf16=1", "opt=adam")
    ref = _single_process("adam")
    for k in ref:
        assert torch.equal(res[0]["state"][k], res[1]["state"][k])
        torch.testing.assert_close(res[0]["state"][k], ref[k], atol=5e-3, rtol=0)


def test_multiworker_from_tf_config(tmp_path):
    ports = free_ports(2)
    cluster = {"worker": [f"127.0.0.1:{p}" for p in ports]}

    def env(r):
        return {"TF_CONFIG": json.dumps({"cluster": cluster, "task": {"type": "worker",
                                                                      "index": r}}),
                "RANK": None, "WORLD_SIZE": None, "LOCAL_RANK": None, "MASTER_ADDR": None,
                "MASTER_PORT": None}
    res = _launch("multiworker", 2, tmp_path, extra_env=env)
    _assert_replicas(res, _single_process())


@pytest.mark.parametrize("num_ps", [1, 2])
def test_colocated_parameter_server_sync(tmp_path, num_ps):
    res = _launch("colocated_ps", 2, tmp_path, f"num_ps={num_ps}", "opt=adam")
    _assert_replicas(res, _single_process("adam"), atol=2e-5)   # Adam normalises fp noise


def test_colocated_ps_sharded_owners_reduce_scatter(tmp_path):
    """num_ps == world with an elementwise optimizer: every rank owns an equal chunk of every
    bucket (reduce-scatter push from the backward hooks, all-gather pull overlapped with the
    next forward); many buckets + the direct flat-buffer gradient writes of the native ops."""
    res = _launch("colocated_ps", 2, tmp_path, "num_ps=2", "bucket_mb=0.05", "direct=1",
                  "opt=momentum")
    assert all(r["sharded"] is True for r in res)
    _assert_replicas(res, _single_process("momentum"))
    off = _launch("colocated_ps", 2, tmp_path, "num_ps=2", "overlap=0", "opt=momentum")
    _assert_replicas(off, _single_process("momentum"))


def test_colocated_ps_bert_fenced_against_overlapped_gathers(tmp_path):
    """every ops entry point that reads a variable waits for its bucket's
    overlapped all-gather.  A tiny BERT (dense, fused bias + GELU + dense, LayerNorm, embeddings)
    on the sharded colocated PS trains identically with the gathers overlapped and serial, and
    the replicas agree in both."""
    on = _launch("colocated_bert", 2, tmp_path, "steps=4", "overlap=1")
    off = _launch("colocated_bert", 2, tmp_path, "steps=4", "overlap=0")
    assert all(r["sharded"] is True for r in on + off)
    for k in on[0]["state"]:
        assert torch.equal(on[0]["state"][k], off[0]["state"][k]), k
        assert torch.equal(on[0]["state"][k], on[1]["state"][k]), k
    assert on[0]["loss"] == off[0]["loss"]


def test_colocated_ps_lamb_keeps_variable_aligned_owners(tmp_path):
    """LAMB's per-tensor trust ratio cannot be split between owners: owner ranges stay on
    variable boundaries (reduce / broadcast path) and still match one process."""
    res = _launch("colocated_ps", 2, tmp_path, "num_ps=2", "opt=lamb")
    assert all(r["sharded"] is False for r in res)
    _assert_replicas(res, _single_process("lamb"), atol=2e-5)


@pytest.mark.parametrize("kind,args", [("mirrored", ()), ("colocated_ps", ("num_ps=1",)),
                                       ("colocated_ps", ("bucket_mb=0.05", "direct=1"))],
                         ids=["mirrored", "ps", "ps_many_buckets"])
def test_forced_reducer_one_rank_is_bit_identical(tmp_path, kind, args):
    """DTF_FORCE_REDUCER=1: a one-rank world still builds the process group and the
    communicating reducer (hooks, collectives, finish, owner apply, overlapped gathers); the
    result must equal the plain single-process run bit for bit."""
    res = _launch(kind, 1, tmp_path, *args, extra_env=lambda r: {"DTF_FORCE_REDUCER": "1"})
    assert res[0]["reducer"] in ("BucketedAllReduce", "_ColocatedPSReducer")
    assert all(e >= 1 for e, _ in res[0]["early_launches"])
    plain = _launch(kind, 1, tmp_path, *args, extra_env=lambda r: {"DTF_FORCE_REDUCER": "0"})
    assert plain[0]["reducer"] == "_NullReducer"
    for k, v in plain[0]["state"].items():
        assert torch.equal(res[0]["state"][k], v), k


def test_colocated_ps_collective_checkpoint_and_restore(tmp_path):
    """Sharded parameter server + MonitoredTrainingSession on both ranks: the step-triggered
    save is collective (slot chunks gathered from their owners), so the chief's checkpoint holds
    the SAME Adam slots as a one-process run; a new session restores on the chief and every
    rank receives the restored variables, slots, update count and global step."""
    res = _launch("colocated_ckpt", 2, tmp_path, "num_ps=2", "opt=adam")
    assert all(r["sharded"] is True for r in res)
    ref_state, ref_opt = _single_process("adam", with_opt=True)
    from distributedtensorflow_amd.train.checkpoint import latest_checkpoint, load_variable
    last = latest_checkpoint(str(tmp_path / "ckpt"))
    assert last.endswith("model.ckpt-3"), last
    import numpy as np
    for name, t in ref_opt.slot_variables().items():
        got = load_variable(last, name)
        want = t.detach()
        if getattr(next(p for p in ref_opt.space.order
                        if name.startswith(p._dtf_name + "/")), "_dtf_layout", None) == "KRSC":
            want = want.permute(1, 2, 3, 0)
        elif want.dim() == 2:
            want = want.t()
        np.testing.assert_allclose(got, want.numpy(), atol=2e-6, rtol=1e-4, err_msg=name)
    r0, r1 = res[0]["restored"], res[1]["restored"]
    assert torch.equal(r0["master"], r1["master"])
    for a, b in zip(r0["slots"], r1["slots"]):
        assert torch.equal(a, b)
    assert r0["iterations"] == r1["iterations"] == 3
    assert r0["global_step"] == r1["global_step"] == 3


# ----------------------------------------------------------------------------- between-graph PS
@pytest.fixture(scope="module")
def mnist_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("mnist")
    from distributedtensorflow_amd.data import mnist
    mnist.load_arrays(str(d), "train")          # writes the offline synthetic stand-in once
    return str(d)


def _ps_run(tmp_path, mnist_dir, num_ps, num_workers, steps, *flags):
    codes, logs = launch_local(os.path.join(ROOT, "run_mnist_distributed.py"), num_ps,
                               num_workers, str(tmp_path),
                               [f"--max_steps={steps}", f"--data_dir={mnist_dir}",
                                f"--log_dir={tmp_path}/tb", "--batch_size=32", *flags],
                               env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2"}, timeout_s=300)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-2000:] for k, t in text.items()}
    return text


def test_between_graph_async_ps(tmp_path, mnist_dir):
    text = _ps_run(tmp_path, mnist_dir, 1, 2, 30)
    chief = text["worker0"]
    lines = re.findall(r"Worker \(0\): loss = ([0-9.]+) \(global step: (\d+)\)", chief)
    assert lines, chief[-2000:]
    steps = [int(s) for _, s in lines]
    assert steps == sorted(steps) and steps[-1] >= 30
    assert float(lines[-1][0]) < float(lines[0][0])
    assert "Close Parameter Server" in text["ps0"]
    from distributedtensorflow_amd.summary.events import read_scalars
    tb = [os.path.join(dp, ) for dp, _, fs in os.walk(tmp_path / "tb") if fs]
    assert tb and "Loss" in read_scalars(tb[0])


def test_between_graph_sync_replicas_two_ps(tmp_path, mnist_dir):
    text = _ps_run(tmp_path, mnist_dir, 2, 2, 12, "--sync_replicas")
    lines = re.findall(r"global step: (\d+)\)", text["worker0"])
    steps = [int(s) for s in lines]
    # synchronous aggregation: every applied update consumed both workers' gradients, so the
    # chief sees each global step at most once and the run ends at max_steps
    assert len(set(steps)) == len(steps) and steps[-1] >= 12
    assert "Close Parameter Server" in text["ps0"] and "Close Parameter Server" in text["ps1"]


def test_heartbeat_detects_silent_peer(tmp_path):
    port = free_ports(1)[0]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"),
                                       "heartbeat", str(tmp_path)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = [p.communicate(timeout=120)[0].decode() for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    res = json.load(open(tmp_path / "hb.json"))
    assert res["failed"] == [1] and res["after_s"] < 8


def test_allreduce_bandwidth_tool_gloo(tmp_path):
    """tools/allreduce_bw.py (SURVEY §5.8 bus-bandwidth sweep) runs under torchrun, 2 ranks."""
    port = free_ports(1)[0]
    out = tmp_path / "bw.jsonl"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "tools", "allreduce_bw.py"), "--min-mb", "0.25",
                        "--max-mb", "0.5", "--iters", "2", "--warmup", "1", "--bucket-mb", "64",
                        "--out", str(out)],
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2"),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = [json.loads(line) for line in open(out)]
    assert [x["size_mb"] for x in rows[:-1]] == [0.25, 0.5]
    assert all(x["busbw_GBps"] > 0 for x in rows[:-1]) and rows[-1]["bucketed_allreduce_ms"] > 0


@pytest.mark.parametrize("victim", ["worker:1", "worker:0"], ids=["worker", "chief"])
def test_any_task_killed_is_restarted_and_training_resumes(tmp_path, mnist_dir, victim):
    """Recovery from ANY task's death (reference run_mnist_distributed.py:128-132,
    146 and the Supervisor's retrying non-chiefs, templates/00_mnist_replica.py:196-211): the
    launcher hosts the rendezvous store, so a non-chief worker OR the chief can die (SIGKILL at
    global step 20).  The launcher bumps the cluster epoch and restarts it as a fresh process;
    the surviving worker re-forms the cluster in the new epoch, the PS task leaves and is
    restarted for it (its shard is re-seeded), the chief -- surviving or restarted -- restores
    the latest checkpoint into the new PS, and training reaches max_steps with a consistent
    global step in the final checkpoint."""
    ckpt = tmp_path / "ckpt"
    codes, logs = launch_local(os.path.join(ROOT, "run_mnist_distributed.py"), 1, 2,
                               str(tmp_path),
                               ["--max_steps=45", f"--data_dir={mnist_dir}",
                                f"--log_dir={tmp_path}/tb", "--batch_size=32",
                                f"--checkpoint_dir={ckpt}", "--save_checkpoint_steps=10"],
                               env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2",
                                    "DTF_FAULT_SIGKILL": f"{victim}@20"},
                               timeout_s=300, max_restarts=1)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-3000:] for k, t in text.items()}
    dead = "worker" + victim.split(":")[1]
    alive = "worker1" if dead == "worker0" else "worker0"
    assert "restarting (1/1), cluster epoch 1" in text[dead], text[dead][-2000:]
    assert "fault injection: SIGKILL" in text[dead]
    assert "recovered: generation 1" in text[alive], text[alive][-3000:]
    assert "rejoining the new cluster epoch" in text["ps0"]
    if dead == "worker0":      # the restarted chief restored the checkpoint on creation
        assert text["worker0"].count("run main with args") == 2
    from distributedtensorflow_amd.train.checkpoint import latest_checkpoint, load_variable
    last = latest_checkpoint(str(ckpt))
    # async training: as with TF's CheckpointSaverHook, the file is named by the global step the
    # chief read, and the other worker may push (advance the step) before the variables are read
    named, saved = int(last.rsplit("-", 1)[1]), int(load_variable(last, "global_step"))
    assert named >= 45 and 0 <= saved - named <= 2, (last, saved)
    steps = [int(s) for s in re.findall(r"global step: (\d+)\)", text["worker0"])]
    # async: the other worker may take the last two steps while the chief is between steps, and
    # a pipelined step reports a lower bound of the step its push became (one step in flight)
    assert steps and steps[-1] >= 42, steps[-5:]


@pytest.mark.parametrize("strategy", ["mirrored", "ps"])
def test_collective_rank_killed_world_reforms_and_resumes(tmp_path, strategy):
    """A 2-rank synchronous world (MirroredStrategy, or the sharded colocated parameter server)
    under launch_collective: rank 1 is SIGKILLed at step 5.  The launcher restarts it alone in a
    new epoch; rank 0's collective fails (CommError), it leaves the broken group, joins the new
    epoch, rebuilds its reducer, restores the chief's latest checkpoint (step 3) and broadcasts
    it; both ranks reach step 12 bit-identical."""
    from distributedtensorflow_amd.cluster.launcher import launch_collective
    codes, logs = launch_collective(os.path.join(HERE, "dist_worker.py"), 2, str(tmp_path),
                                    ["mirrored_recovery", str(tmp_path), "steps=12", "save=3",
                                     f"strategy={strategy}", "opt=adam"],
                                    env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2",
                                         "DTF_FAULT_SIGKILL": "rank:1@5"},
                                    timeout_s=240, max_restarts=1)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-3000:] for k, t in text.items()}
    assert "restarting (1/1), cluster epoch 1" in text["rank1"]
    assert "recovered: generation 1" in text["rank0"], text["rank0"][-3000:]
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    assert res[0]["recoveries"] == 1 and res[1]["restart"] == 1
    assert all(r["global_step"] == 12 for r in res)
    assert res[0]["fingerprints"] == res[1]["fingerprints"]
    for k in res[0]["state"]:
        assert torch.equal(res[0]["state"][k], res[1]["state"][k]), k


@pytest.mark.parametrize("pipeline", ["0", "1"], ids=["serial", "pipelined"])
def test_ps_killed_mid_run_is_restarted_and_training_resumes(tmp_path, mnist_dir, pipeline):
    """Real failure recovery (reference run_mnist_distributed.py:146): the PS task
    dies (SIGKILL at global step 25, DTF_FAULT_KILL_PS_AT_STEP), the launcher restarts it as a
    fresh process, every task joins the next process-group generation, the chief restores the
    latest checkpoint (variables + Adam slots + step) into the new PS, training reaches
    max_steps and the final checkpoint is consistent with the final global step."""
    ckpt = tmp_path / "ckpt"
    codes, logs = launch_local(os.path.join(ROOT, "run_mnist_distributed.py"), 1, 2,
                               str(tmp_path),
                               ["--max_steps=45", f"--data_dir={mnist_dir}",
                                f"--log_dir={tmp_path}/tb", "--batch_size=32",
                                f"--checkpoint_dir={ckpt}", "--save_checkpoint_steps=10"],
                               env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2",
                                    "DTF_FAULT_KILL_PS_AT_STEP": "25",
                                    "DTF_PS_PIPELINE": pipeline,
                                    # every recovery wait bounded well below the job budget
                                    "DTF_RECOVERY_TIMEOUT_S": "60", "DTF_PS_TIMEOUT_S": "60"},
                               timeout_s=300, max_ps_restarts=1)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-3000:] for k, t in text.items()}
    assert "restarting (1/1)" in text["ps0"]                    # the PS really died once
    assert text["ps0"].count("Started Parameter Server") == 2
    for w in ("worker0", "worker1"):
        assert "recovered: generation 1" in text[w], text[w][-3000:]
    # the chief restored a checkpoint taken before the crash (every ~10 async global steps)
    m = re.search(r"restored=(\S+model\.ckpt-(\d+))", text["worker0"])
    assert m and 10 <= int(m.group(2)) <= 25, text["worker0"][-3000:]
    steps = [int(s) for s in re.findall(r"global step: (\d+)\)", text["worker0"])]
    assert steps[-1] >= 42, steps[-5:]      # async + pipelined: see the test above
    from distributedtensorflow_amd.train.checkpoint import latest_checkpoint, load_variable
    last = latest_checkpoint(str(ckpt))
    # async training: as with TF's CheckpointSaverHook, the file is named by the global step the
    # chief read, and the other worker may push (advance the step) before the variables are read
    named, saved = int(last.rsplit("-", 1)[1]), int(load_variable(last, "global_step"))
    assert named >= 45 and 0 <= saved - named <= 2, (last, saved)
    assert abs(load_variable(last, "conv2d/kernel/Adam")).sum() > 0     # slots survived



def test_bench_ps_async_flow_cpu(tmp_path):
    """bench.py --strategy ps_async (BASELINE config 4 in the reference's async mode): the bench
    process launches 1 PS + 2 worker tasks, every push is applied on arrival (no drops), and
    the rank-0 style JSON line carries the aggregate and the push/wait/pull breakdown."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--strategy", "ps_async",
                        "--num-workers", "2", "--batch", "2", "--image-size", "32", "--steps",
                        "2", "--warmup", "1", "--timeout", "200"],
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2"),
                       capture_output=True, text=True, timeout=260, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = rec["config"]
    assert cfg["parallelism"] == "ps1+async2" and cfg["data_plane"] == "shm"
    assert cfg["ps_applied"] == cfg["ps_pushes"] == 2 * (2 + 1)       # nothing dropped
    assert cfg["final_global_step"] == 6 and rec["value"] > 0
    assert set(cfg["worker_host_ms_per_step"]) == {"copy_sync_ms_per_step", "wait_ms_per_step",
                                                   "pull_ms_per_step", "fence_ms_per_step",
                                                   "answer_ms_per_step"}
    # the /dev/shm plane on CPU runs the pipelined push/pull state machine too (CPU stand-ins for
    # the side stream and its events)
    assert cfg["pipelined_push_pull"] is True


@pytest.mark.parametrize("kind,args", [("mirrored", ("bucket_mb=0.05",)),
                                       ("colocated_ps", ("num_ps=8", "bucket_mb=0.05")),
                                       ("colocated_ps", ("num_ps=1", "bucket_mb=0.05"))],
                         ids=["mirrored", "sharded_ps", "one_ps"])
def test_eight_ranks_match_single_process(tmp_path, kind, args):
    """The driver's N = 8 layout rehearsed on gloo: 8 ranks (2 images each of the 16-image
    global batch), many buckets; the sharded parameter server splits every bucket 8 ways, and
    BASELINE config 4's "1 PS + 8 workers" keeps every variable on rank 0 (owner plan: one
    range, owner 0, covering the whole flat buffer)."""
    res = _launch(kind, 8, tmp_path, *args, timeout=300)
    if kind == "colocated_ps":
        assert all(r["sharded"] is (args[0] == "num_ps=8") for r in res)
        if args[0] == "num_ps=1":
            for rec in res:
                owners = {o for o, _, _ in rec["ranges"]}
                assert owners == {0}, rec["ranges"]
                ends = sorted((s, e) for _, s, e in rec["ranges"])
                assert all(a[1] == b[0] for a, b in zip(ends, ends[1:]))   # contiguous cover
    _assert_replicas(res, _single_process(), atol=5e-6)
    # every rank: the same bucket plan, the same collective issue order (checked collectively by
    # verify_bucket_agreement inside the run, and here from the saved records)
    assert all(r["plan"] == res[0]["plan"] and r["order"] == res[0]["order"] for r in res)
    assert len(res[0]["plan"]["buckets"]) >= 4 and sorted(res[0]["order"]) == \
        list(range(len(res[0]["plan"]["buckets"])))
    assert all(r["agreement"] == res[0]["agreement"] for r in res)
    if kind == "colocated_ps" and args[0] == "num_ps=8":
        # reduce-scatter / all-gather chunk offsets = the sharded owner plan at every rank:
        # rank r owns chunk r of every bucket, equal chunks that tile the bucket exactly
        for r, rec in enumerate(res):
            for b, (s, e, _) in enumerate(rec["plan"]["buckets"]):
                c = (e - s) // 8
                assert [list(p) for p in rec["plan"]["pieces"][b]] == \
                    [[o, s + o * c, s + (o + 1) * c] for o in range(8)]
                assert list(rec["ranges"][b]) == [r, s + r * c, s + (r + 1) * c]


def test_forced_bucket_order_mismatch_fails_within_the_deadline(tmp_path):
    """A rank that issues its bucket collectives in another order (DTF_DEBUG_PERTURB_BUCKET_ORDER)
    sums the wrong buckets or blocks: the run must fail -- by the order check or by the comm
    watchdog's deadline -- quickly and loudly, never train on silently or hang."""
    import time
    t0 = time.time()
    with pytest.raises(AssertionError) as ei:
        _launch("mirrored", 2, tmp_path, "bucket_mb=0.05", timeout=120,
                extra_env=lambda r: {"DTF_DEBUG_PERTURB_BUCKET_ORDER": "1",
                                     "DTF_COMM_TIMEOUT_S": "5"})
    assert time.time() - t0 < 90
    msg = str(ei.value)
    assert "collective order differs" in msg or "CommError" in msg or "did not complete" in msg, \
        msg[-3000:]


def test_bench_ps_async_eight_workers_cpu(tmp_path):
    """BASELINE config 4's shape in the reference's own async mode, rehearsed on the CPU: 1 PS +
    8 worker tasks launched by bench.py, every push applied (Hogwild, no drops), the global step
    counts all 8 workers' pushes, and the JSON names every worker's device (on a GPU node the
    plan is cuda:0..7 with the PS on cuda:0: tests/test_bench_integrity.py)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--strategy", "ps_async",
                        "--num-workers", "8", "--batch", "2", "--image-size", "32", "--steps",
                        "2", "--warmup", "1", "--timeout", "400"],
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1"),
                       capture_output=True, text=True, timeout=460, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = rec["config"]
    assert cfg["parallelism"] == "ps1+async8" and len(cfg["worker_devices"]) == 8
    assert cfg["ps_applied"] == cfg["ps_pushes"] == 8 * (2 + 1)
    assert cfg["final_global_step"] == 8 * 3
    assert rec["n_gpus"] == 0 and cfg["ps_device"] is None        # CPU host: no devices used
    assert cfg["dtf_env"] == {k: v for k, v in sorted(os.environ.items())
                              if k.startswith("DTF_")}
