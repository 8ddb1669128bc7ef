"""Bounded collective waits (VERDICT r3 "Next round" item 2).

The reference recovers from a dead task because TF1's MonitoredTrainingSession recreates its
session on AbortedError/UnavailableError (/root/reference/run_mnist_distributed.py:128-132,146).
A GPU collective world only gets there if a survivor blocked on a dead peer is RELEASED: these
tests pin the watchdog that does it (parallel/watchdog.py) -- a stalled collective trips it within
its deadline, the trip runs the communicators' abort callbacks, and every later issue / step check
raises CommError (recoverable under the launcher, a loud failure otherwise)."""
import json
import os
import subprocess
import sys
import threading
import time

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_stalled_collective_trips_within_deadline_and_aborts():
    from distributedtensorflow_amd.parallel.strategy import CommError
    from distributedtensorflow_amd.parallel.watchdog import CommWatchdog
    wd = CommWatchdog(timeout_s=0.4, interval_s=0.02)
    released = threading.Event()        # the "RCCL kernel": completes only when aborted
    wd.add_abort(released.set)
    t0 = time.monotonic()
    wd.watch(released.is_set, "fake all_reduce")
    assert wd.wait_tripped(5.0)
    dt = time.monotonic() - t0
    assert 0.4 <= dt < 1.5, dt
    assert released.is_set()            # abort ran: the blocked collective is released
    assert "fake all_reduce" in wd.failed and "DTF_COMM_TIMEOUT_S" in wd.failed
    with pytest.raises(CommError, match="watchdog"):
        wd.check()
    wd.stop()


def test_completed_collectives_never_trip():
    from distributedtensorflow_amd.parallel.watchdog import CommWatchdog
    wd = CommWatchdog(timeout_s=0.3, interval_s=0.02)
    aborted = []
    wd.add_abort(lambda: aborted.append(1))
    for _ in range(50):
        wd.watch(lambda: True, "done")
    time.sleep(0.6)
    assert wd.failed is None and not aborted and wd.inflight() == 0
    wd.check()
    wd.stop()


def test_probe_failure_trips_immediately_and_late_abort_runs():
    """An epoch bump / async RCCL error trips the watchdog with nothing in flight; a communicator
    registered after the trip is aborted at registration."""
    from distributedtensorflow_amd.parallel.watchdog import CommWatchdog
    wd = CommWatchdog(timeout_s=100, interval_s=0.02)
    flag = threading.Event()
    wd.add_probe(lambda: "cluster epoch moved" if flag.is_set() else None)
    time.sleep(0.1)
    assert wd.failed is None
    flag.set()
    assert wd.wait_tripped(2.0) and wd.failed == "cluster epoch moved"
    late = []
    wd.add_abort(lambda: late.append(1))
    assert late == [1]
    wd.stop()


def test_errored_work_trips():
    from distributedtensorflow_amd.parallel.watchdog import CommWatchdog
    wd = CommWatchdog(timeout_s=100, interval_s=0.02)

    def boom():
        raise RuntimeError("NCCL error: remote process exited")
    wd.watch(boom, "c10d all_reduce")
    assert wd.wait_tripped(2.0) and "remote process exited" in wd.failed
    wd.stop()


def test_rccl_uid_key_restarts_with_each_world():
    """a restarted rank and the survivors must agree on the unique-id store key."""
    from distributedtensorflow_amd.parallel import comm
    comm.reset_uid_index()
    assert comm._next_uid_key() == "dtf/rccl_uid/0"
    assert comm._next_uid_key() == "dtf/rccl_uid/1"
    comm.reset_uid_index()               # what init_process_group_from_env does per world
    assert comm._next_uid_key() == "dtf/rccl_uid/0"


def test_session_refuses_to_continue_after_trip(monkeypatch):
    """A step whose collective was aborted must not reach the hooks (the checkpoint saver)."""
    from distributedtensorflow_amd.parallel import watchdog
    from distributedtensorflow_amd.parallel.strategy import CommError
    from distributedtensorflow_amd.train.session import MonitoredTrainingSession
    wd = watchdog.reset_watchdog()
    try:
        sess = MonitoredTrainingSession(checkpoint_dir=None, save_checkpoint_secs=None,
                                        save_summaries_steps=None, log_step_count_steps=None)
        seen = []

        def step():
            wd.trip("injected: peer died mid-step")
            seen.append(1)
            return 1
        with pytest.raises(CommError, match="peer died"):
            sess.run(step)
        assert seen == [1]
    finally:
        watchdog.reset_watchdog()


def test_hung_peer_flagged_in_two_rank_gloo_world(tmp_path):
    """2 ranks on gloo; rank 1 stays alive but never enters the all-reduce.  Rank 0's watchdog
    flags the collective within DTF_COMM_TIMEOUT_S (2 s) and the next issue raises CommError."""
    from distributedtensorflow_amd.cluster.launcher import free_ports
    port = free_ports(1)[0]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1",
                   PYTHONPATH=ROOT, DTF_COMM_TIMEOUT_S="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"),
                                       "hung_peer", str(tmp_path)], env=env,
                                      stdout=open(tmp_path / f"r{r}.log", "w"),
                                      stderr=subprocess.STDOUT))
    try:
        for p in procs:
            p.wait(timeout=120)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert procs[0].returncode == 0, open(tmp_path / "r0.log").read()[-3000:]
    res = json.load(open(tmp_path / "wd.json"))
    assert res["tripped"], res
    assert 2.0 <= res["after_s"] < 8.0, res
    assert res["error"] and "watchdog" in res["error"], res


def test_bench_refuses_more_gpus_than_visible(tmp_path):
    """bench.py never measures fewer GPUs than asked: --gpus 2 with fewer visible devices exits
    non-zero quickly with the device-count message (here: a CPU box, 0 devices)."""
    if torch.cuda.device_count() >= 2:
        pytest.skip("this box has >= 2 GPUs")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "1"], env=env, capture_output=True,
                       text=True, timeout=120, cwd=ROOT)
    assert p.returncode != 0
    assert "refusing to measure fewer GPUs" in p.stderr, p.stderr[-2000:]
    assert time.time() - t0 < 60


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "1"], env=env, capture_output=True,
                       text=True, timeout=120, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr, p.stderr[-2000:]


def _fake_rccl(rank, world):
    """An RcclComm whose kernel calls are recorded instead of issued (no GPU / RCCL needed)."""
    from distributedtensorflow_amd.parallel.comm import RcclComm
    from distributedtensorflow_amd.parallel.watchdog import CommWatchdog

    class K:
        calls = []

        def __getattr__(self, name):
            return lambda *a: K.calls.append((name, a))
    c = object.__new__(RcclComm)
    c.K, c.rank, c.world, c.comm = K(), rank, world, 1
    c.wd = CommWatchdog(timeout_s=100)
    c._issue = lambda fn, *t, what="": fn(c.comm, 0)
    return c, K.calls


def test_rccl_in_place_rules_of_the_sharded_ps():
    """The colocated PS reduce-scatters / all-gathers IN PLACE on flat-buffer views.  NCCL
    defines in-place only for recvbuff == sendbuff + rank * count (reduce-scatter) and sendbuff ==
    recvbuff + rank * count (all-gather); at world 1 every layout passes, so the rule is checked
    on the host for world 8: the reducer's layout is accepted at every rank, a shifted one is
    refused."""
    W, c = 8, 96
    g = torch.zeros(4 * W * c)
    s = 64                                      # a bucket starting inside the flat buffer
    bucket = g[s:s + W * c]
    for r in range(W):
        comm, calls = _fake_rccl(r, W)
        comm.reduce_scatter(g[s + r * c:s + (r + 1) * c], bucket)
        comm.all_gather(bucket, g[s + r * c:s + (r + 1) * c])
        assert [n for n, _ in calls] == ["rccl_reduce_scatter", "rccl_all_gather"]
    comm, _ = _fake_rccl(3, W)
    with pytest.raises(ValueError, match="chunk 3"):
        comm.reduce_scatter(g[s + 2 * c:s + 3 * c], bucket)
    with pytest.raises(ValueError, match="chunk 3"):
        comm.all_gather(bucket, g[s + 4 * c:s + 5 * c])
    comm.reduce_scatter(torch.zeros(c), bucket)            # disjoint buffers: always fine


def test_ps_peer_access_check(monkeypatch):
    """A worker mapping an owner's HBM shard on ANOTHER GPU needs peer access: checked up front
    with hipDeviceCanAccessPeer and refused with the reason (VERDICT r3 missing #3)."""
    from distributedtensorflow_amd.parallel import ps_device
    desc = {"master": {"kind": "ipc"}, "device": 3}
    calls = []

    def can(a, b):
        calls.append((a, b))
        return False
    monkeypatch.setattr(torch.cuda, "can_device_access_peer", can)
    ps_device.check_peer_access(desc, torch.device("cuda", 3))          # same GPU: no query
    assert calls == []
    with pytest.raises(RuntimeError, match="hipDeviceCanAccessPeer"):
        ps_device.check_peer_access(desc, torch.device("cuda", 5))
    assert calls == [(5, 3)]
    monkeypatch.setattr(torch.cuda, "can_device_access_peer", lambda a, b: True)
    ps_device.check_peer_access(desc, torch.device("cuda", 5))
    ps_device.check_peer_access({"master": {"kind": "shm"}, "device": None}, torch.device("cpu"))


def test_ps_bucket_plan_covers_the_flat_buffer():
    from distributedtensorflow_amd.parallel.ps_strategy import _bucket_plan

    class Space:
        offsets = [0, 64, 1088, 5184, 5248]
        numel = 9344
        order = [None] * 5
    plan = _bucket_plan(Space, 4096)                 # 1024-float buckets
    assert plan[0][0] == 0 and plan[-1][1] == Space.numel
    assert all(a[1] == b[0] for a, b in zip(plan, plan[1:]))
    assert sorted(i for _, _, m in plan for i in m) == list(range(5))


def test_hung_rank_ends_the_job_loudly(tmp_path):
    """No restarts configured and rank 1 hangs mid-run: rank 0's collective fails within
    DTF_COMM_TIMEOUT_S, rank 0 exits non-zero, and the launcher stops the hung rank -- the job
    ends in well under the launcher's own timeout instead of hanging."""
    from distributedtensorflow_amd.cluster.launcher import launch_collective
    t0 = time.time()
    codes, logs = launch_collective(os.path.join(HERE, "dist_worker.py"), 2, str(tmp_path),
                                    ["hang_mid_run", str(tmp_path), "at=4"],
                                    env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1",
                                         "DTF_COMM_TIMEOUT_S": "4"},
                                    timeout_s=150, max_restarts=0)
    took = time.time() - t0
    text = {k: open(v).read() for k, v in logs.items()}
    assert codes[0] != 0 and codes[1] != 0, (codes, text["rank0"][-2000:])
    assert "rank 1 hangs" in text["rank1"]
    assert "failed for good" in text["rank1"]
    assert took < 90, took


def test_watchdog_aborts_a_communicator_blocked_inside_an_enqueue():
    """the native communicator is a blocking one, so an enqueue can wait inside RCCL
    on a dead peer.  The watchdog must still probe it, trip on the collective's deadline (which
    is registered before the enqueue) and call ncclCommAbort -- which releases the blocked
    enqueue, whose caller then gets CommError -- without waiting for that enqueue."""
    import threading

    from distributedtensorflow_amd.parallel.comm import RcclComm
    from distributedtensorflow_amd.parallel.strategy import CommError
    from distributedtensorflow_amd.parallel.watchdog import CommWatchdog

    entered, released, log = threading.Event(), threading.Event(), []

    class K:
        def rccl_async_error(self, comm):
            log.append(("probe", comm))
            return 0

        def rccl_comm_destroy(self, comm, abort):
            log.append(("destroy", comm, abort))
            released.set()                       # ncclCommAbort unblocks the stuck enqueue

        def rccl_all_reduce(self, comm):
            entered.set()
            assert released.wait(20), "enqueue never released"

    c = object.__new__(RcclComm)
    c.K, c.comm, c._lock, c._inuse = K(), 77, threading.Lock(), 0
    c.wd = CommWatchdog(timeout_s=0.5, interval_s=0.02)
    c.wd.add_abort(c.abort)
    c.wd.add_probe(c._probe)
    err = []

    def issue():
        try:
            c._enqueue(lambda comm, st: c.K.rccl_all_reduce(comm), 0, "all_reduce")
        except CommError as e:
            err.append(e)

    t = threading.Thread(target=issue, daemon=True)
    t.start()
    assert entered.wait(5)
    n_probes = sum(1 for e in log if e[0] == "probe")
    time.sleep(0.1)
    # the probe keeps running while the enqueue is blocked (it never waits on the enqueue)
    assert sum(1 for e in log if e[0] == "probe") > n_probes
    assert c.wd.wait_tripped(10), "the blocked enqueue never tripped the deadline"
    assert "all_reduce did not complete" in c.wd.failed
    t.join(10)
    assert not t.is_alive()
    assert ("destroy", 77, 1) in log and c.comm == 0 and c._inuse == 0
    assert err and "aborted during the all_reduce enqueue" in str(err[0])
    with pytest.raises(CommError):
        c._enqueue(lambda comm, st: None, 0, "broadcast")
