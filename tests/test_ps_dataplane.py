"""Parameter-server data plane (parallel/ps_device.py + csrc/native/shm_ctl.cpp).

Every case runs on BOTH planes: ``cpu`` (the owner shard in /dev/shm) and ``cuda`` (the owner
shard in HBM exported through hipIpc, the owner's applies on its own HIP streams; marked
``gpu``).  Workers write gradients into their mailbox slot, post, and the owner's service
thread applies TF-exact Adam on arrival (async) or after ``replicas_to_aggregate`` fresh
gradients (SyncReplicasOptimizer, stale ones dropped) — reference
``run_mnist_distributed.py:107-116``, ``templates/00_mnist_replica.py:168-191``.  The results
are compared with numpy-style oracles of TF's update formulas, so an apply on the wrong slot, a
missing 1/N scale or a lost first gradient fails the test."""
import threading
import time

import pytest
import torch

from distributedtensorflow_amd.optimizers.base import FlatSpace, tf_adam_lr_t
from distributedtensorflow_amd.parallel import ps_device
from distributedtensorflow_amd.parallel.ps_service import choose_plane


DEV = "cpu"


@pytest.fixture(params=["cpu", pytest.param("cuda", marks=pytest.mark.gpu)], autouse=True)
def plane_device(request):
    """Run each data-plane case on the /dev/shm plane and on the HBM + hipIpc plane."""
    global DEV
    if request.param == "cuda" and not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    DEV = request.param
    yield request.param
    DEV = "cpu"


def _space(seed=0):
    g = torch.Generator().manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(*s, generator=g).to(DEV)) for s in
          [(5, 5, 1, 32), (32,), (70, 33), (33,), (10,)]]
    for i, p in enumerate(ps):
        p._dtf_name = f"v{i}"
    sp = FlatSpace(ps)
    return sp, ps


def _rand_grad(space):
    """Random gradient on the variables, zero on the alignment padding (never transferred)."""
    g = torch.zeros(space.numel)
    for v, o in zip(space.order, space.offsets):
        g[o:o + v.numel()] = torch.randn(v.numel())
    return g.to(DEV)


def _owner(space, plan, sync=False, r2a=None, workers=(1, 2), opt=None):
    spec = ps_device.spec_for(space, plan)
    spec.update({"optimizer": opt or {"type": "adam", "learning_rate": 0.01, "beta1": 0.9,
                                      "beta2": 0.999, "epsilon": 1e-8},
                 "sync": sync, "replicas_to_aggregate": r2a, "global_step": 0})
    vals = torch.cat([space.order[i].detach().reshape(-1) for i in plan["vars"]]).cpu()
    sh = ps_device.OwnerShard(spec, vals, DEV, list(workers), 0)
    sh.start()
    return sh


def _links(sh, plan, spaces):
    d = sh.descriptor()
    assert d["plane"] == ("ipc" if DEV == "cuda" else "shm")
    return [ps_device.PSLink(d, plan, w, DEV, 0, timeout_s=10) for w in range(len(spaces))]


def _push(link, space):
    """Worker side of a push: gradient into the mailbox, device-synchronised, posted."""
    link.copy_grads(space)
    ps_device.sync_device(space.device)


def test_shm_control_roundtrip_and_stop(plane_device):
    if plane_device != "cpu":
        pytest.skip("host-only")
    from distributedtensorflow_amd._lib import _dtf_native as N
    name = f"dtf_t_{time.time_ns()}"
    owner = N.ShmControl(name, True, 3)
    w = N.ShmControl(name, False, 3)
    assert owner.wait_any(10) == []
    w.post(2, 41)
    assert owner.wait_any(100) == [(2, 41)]
    assert w.wait_done(2, 20) is None                      # not answered yet: timeout
    owner.done(2, 7)
    assert w.wait_done(2, 100) == 7
    with pytest.raises(Exception):
        w.post(5, 0)                                        # bad worker index
    w.post(0, 1)
    with pytest.raises(Exception):
        w.post(0, 2)                                        # slot busy until answered
    owner.stop()
    assert owner.wait_any(10) is None
    with pytest.raises(RuntimeError):
        w.wait_done(0, 100)
    del w, owner


def test_shard_plan_balanced_is_one_copy_per_ps(plane_device):
    space, _ = _space()
    plans = ps_device.shard_plan(space, 2, "balanced")
    assert sorted(i for p in plans for i in p["vars"]) == list(range(len(space.order)))
    for p in plans:
        assert len(p["segments"]) == 1                      # contiguous slice -> one copy
    rr = ps_device.shard_plan(space, 2, "round_robin")
    assert rr[0]["vars"] == [0, 2, 4] and rr[1]["vars"] == [1, 3]
    # owner layout reproduces every variable exactly
    for plan in plans + rr:
        owner = torch.zeros(plan["numel"], device=DEV)
        for wo, oo, n in plan["segments"]:
            owner[oo:oo + n] = space.master[wo:wo + n]
        for i, o in zip(plan["vars"], plan["owner_offsets"]):
            v = space.order[i]
            assert torch.equal(owner[o:o + v.numel()], v.detach().reshape(-1))


def test_choose_plane(plane_device):
    if plane_device != "cpu":
        pytest.skip("host-only")
    assert choose_plane("gloo", "cpu") == "gloo"
    assert choose_plane("auto", "cpu") == "shm"
    assert choose_plane("auto", "cuda:0") == "ipc"


def _adam_oracle(p, g, t, lr=0.01, b1=0.9, b2=0.999, eps=1e-8, m=None, v=None):
    m = (1 - b1) * g if m is None else b1 * m + (1 - b1) * g
    v = (1 - b2) * g * g if v is None else b2 * v + (1 - b2) * g * g
    return p - tf_adam_lr_t(lr, b1, b2, t) * m / (v.sqrt() + eps), m, v


def test_async_apply_on_arrival():
    space, _ = _space()
    w_spaces = [_space()[0], _space()[0]]
    plan = ps_device.shard_plan(space, 1)[0]
    sh = _owner(space, plan)
    try:
        links = _links(sh, plan, w_spaces)
        p0 = space.master.clone()
        g0 = _rand_grad(space)
        w_spaces[0].grad.copy_(g0)
        _push(links[0], w_spaces[0])
        links[0].post(0)
        assert links[0].wait() == 1
        links[0].pull(w_spaces[0])
        ref, m, v = _adam_oracle(p0, g0, 1)
        torch.testing.assert_close(w_spaces[0].master, ref, atol=1e-5, rtol=1e-5)
        # second worker's push applies on top (Hogwild: no aggregation, step 2)
        g1 = _rand_grad(space)
        w_spaces[1].grad.copy_(g1)
        _push(links[1], w_spaces[1])
        links[1].post(0)                # computed at a stale step: async applies it anyway
        assert links[1].wait() == 2
        links[1].pull(w_spaces[1])
        ref2, _, _ = _adam_oracle(ref, g1, 2, m=m, v=v)
        torch.testing.assert_close(w_spaces[1].master, ref2, atol=1e-5, rtol=1e-5)
        assert sh.stats["applied"] == 2
    finally:
        err = sh._error
        sh.stop()
        assert err is None, repr(err)


def test_sync_aggregation_stale_drop_and_barrier():
    space, _ = _space()
    w_spaces = [_space()[0], _space()[0]]
    plan = ps_device.shard_plan(space, 1)[0]
    sh = _owner(space, plan, sync=True, r2a=2,
                opt={"type": "sgd", "learning_rate": 0.5, "weight_decay": 0.0})
    try:
        links = _links(sh, plan, w_spaces)
        p0 = space.master.clone()
        g = [_rand_grad(space), _rand_grad(space)]
        for i in range(2):
            w_spaces[i].grad.copy_(g[i])
            _push(links[i], w_spaces[i])
        links[0].post(0)
        time.sleep(0.2)
        assert sh.ctl.state(0) == 2          # TAKEN: held at the token barrier
        res = {}
        t = threading.Thread(target=lambda: res.setdefault(0, links[0].wait()))
        t.start()
        links[1].post(0)
        assert links[1].wait() == 1
        t.join(5)
        assert res[0] == 1
        links[0].pull(w_spaces[0])
        torch.testing.assert_close(w_spaces[0].master, p0 - 0.5 * (g[0] + g[1]) / 2,
                                   atol=1e-5, rtol=1e-5)
        # a gradient computed at step 0 arriving after step 1 closed is stale: dropped at once
        links[1].post(0)
        assert links[1].wait() == 1
        assert sh.stats["dropped_stale"] == 1 and sh.stats["applied"] == 1
    finally:
        err = sh._error
        sh.stop()
        assert err is None, repr(err)


def test_sync_backup_worker_first_arrival_wins():
    space, _ = _space()
    w_spaces = [_space()[0], _space()[0]]
    plan = ps_device.shard_plan(space, 1)[0]
    sh = _owner(space, plan, sync=True, r2a=1,
                opt={"type": "sgd", "learning_rate": 1.0, "weight_decay": 0.0})
    try:
        links = _links(sh, plan, w_spaces)
        p0 = space.master.clone()
        g = _rand_grad(space)
        w_spaces[1].grad.copy_(g)
        _push(links[1], w_spaces[1])
        links[1].post(0)
        assert links[1].wait() == 1              # replicas_to_aggregate=1: closes at once
        _push(links[0], w_spaces[0])
        links[0].post(0)                         # the backup worker's late gradient
        assert links[0].wait() == 1
        links[0].pull(w_spaces[0])
        torch.testing.assert_close(w_spaces[0].master, p0 - g, atol=1e-5, rtol=1e-5)
        assert sh.stats["dropped_stale"] == 1
    finally:
        err = sh._error
        sh.stop()
        assert err is None, repr(err)


def test_stopped_worker_releases_sync_barrier():
    space, _ = _space()
    w_spaces = [_space()[0], _space()[0]]
    plan = ps_device.shard_plan(space, 1)[0]
    sh = _owner(space, plan, sync=True, r2a=2,
                opt={"type": "sgd", "learning_rate": 1.0, "weight_decay": 0.0})
    try:
        links = _links(sh, plan, w_spaces)
        _push(links[0], w_spaces[0])
        links[0].post(0)
        time.sleep(0.1)
        sh.worker_stopped(2)                     # rank of worker 1 (workers=(1, 2))
        assert links[0].wait() == 1
    finally:
        err = sh._error
        sh.stop()
        assert err is None, repr(err)


def test_sync_mean_of_pushed_gradients_every_step():
    """SyncReplicas on the data plane: EVERY step (the first included) applies exactly the mean
    of the two pushed gradients -- the accumulator is cleared and refilled in order on the
    owner's stream (a zero-fill racing the first add would lose a gradient)."""
    space, _ = _space()
    w_spaces = [_space()[0], _space()[0]]
    plan = ps_device.shard_plan(space, 1)[0]
    sh = _owner(space, plan, sync=True, r2a=2,
                opt={"type": "sgd", "learning_rate": 0.25, "weight_decay": 0.0})
    try:
        links = _links(sh, plan, w_spaces)
        p = space.master.clone()
        for step in range(4):
            g = [_rand_grad(space), _rand_grad(space)]
            res = {}
            for i in range(2):
                w_spaces[i].grad.copy_(g[i])
                _push(links[i], w_spaces[i])
            ts = [threading.Thread(target=lambda i=i: (links[i].post(step),
                                                       res.setdefault(i, links[i].wait())))
                  for i in range(2)]
            for th in ts:
                th.start()
            for th in ts:
                th.join(10)
            assert res == {0: step + 1, 1: step + 1}
            p = p - 0.25 * (g[0] + g[1]) / 2
            links[0].pull(w_spaces[0])
            torch.testing.assert_close(w_spaces[0].master, p, atol=1e-5, rtol=1e-5)
        assert sh.stats["applied"] == 4 and sh.stats["aggregated"] == 8
        assert sh.stats["dropped_stale"] == 0
    finally:
        err = sh._error
        sh.stop()
        assert err is None, repr(err)


def test_async_concurrent_pushes_all_applied():
    """Hogwild: both workers post at once; each push is applied exactly once (global step 2),
    and SGD -- additive -- ends at p0 - lr * (g0 + g1) whatever order the applies took."""
    space, _ = _space()
    w_spaces = [_space()[0], _space()[0]]
    plan = ps_device.shard_plan(space, 1)[0]
    sh = _owner(space, plan, opt={"type": "sgd", "learning_rate": 0.5, "weight_decay": 0.0})
    try:
        links = _links(sh, plan, w_spaces)
        p0 = space.master.clone()
        g = [_rand_grad(space), _rand_grad(space)]
        for i in range(2):
            w_spaces[i].grad.copy_(g[i])
            _push(links[i], w_spaces[i])
        links[0].post(0)
        links[1].post(0)
        steps = sorted([links[0].wait(), links[1].wait()])
        assert steps == [1, 2]
        links[0].pull(w_spaces[0])
        torch.testing.assert_close(w_spaces[0].master, p0 - 0.5 * (g[0] + g[1]),
                                   atol=1e-5, rtol=1e-5)
        assert sh.stats["applied"] == 2 and sh.stats["pushes"] == 2
    finally:
        err = sh._error
        sh.stop()
        assert err is None, repr(err)


def test_cross_host_cluster_uses_tcp_plane(plane_device):
    """The device planes map memory between processes of ONE host; a cluster whose tasks are
    on several hosts (config.json by IP, as in the reference) falls back to gloo/TCP."""
    if plane_device != "cpu":
        pytest.skip("host-only")
    from distributedtensorflow_amd.cluster import ClusterSpec
    from distributedtensorflow_amd.parallel.ps_service import PSClient
    local = ClusterSpec({"ps": ["192.168.2.107:8001"], "worker": ["192.168.2.107:6001"]})
    remote = ClusterSpec({"ps": ["10.0.0.1:8001"], "worker": ["10.0.0.2:6001"]})
    assert local.single_host() and not remote.single_host()
    assert ClusterSpec({"ps": ["localhost:1"], "worker": ["127.0.0.1:2"]}).single_host()
    space, _ = _space()
    assert PSClient([0], space=space, data_plane="auto", single_host=True).data_plane == "auto"
    assert PSClient([0], space=space, data_plane="auto", single_host=False).data_plane == "gloo"
    with pytest.raises(ValueError):
        PSClient([0], space=space, data_plane="ipc", single_host=False)
    d = {"host": "some-other-host", "master": {}, "mail": {}}
    with pytest.raises(RuntimeError, match="cannot be"):
        ps_device.PSLink(d, {}, 0, "cpu", 0)


def test_async_applies_of_different_workers_do_not_serialise(plane_device):
    """a Hogwild apply must not queue behind another worker's apply.  Worker 0's
    apply stream is held busy (a long device sleep queued on it first); worker 1's apply, launched
    after it, completes while worker 0's is still pending -- no shard-stream edge orders them."""
    if plane_device != "cuda":
        pytest.skip("device streams")
    space, _ = _space()
    plan = ps_device.shard_plan(space, 1)[0]
    sh = _owner(space, plan, opt={"type": "sgd", "learning_rate": 0.5, "weight_decay": 0.0})
    try:
        with torch.cuda.stream(sh.streams[0]):
            torch.cuda._sleep(400_000_000)            # ~0.2 s of GPU cycles on worker 0's stream
        with sh.lock:
            sh._launch_apply(sh._slot(0), 1.0, 0, [], None)
            sh._launch_apply(sh._slot(1), 1.0, 1, [], None)
        t0 = time.time()
        while not sh.streams[1].query() and time.time() - t0 < 5:
            time.sleep(0.001)
        assert sh.streams[1].query(), "worker 1's apply waited"
        assert not sh.streams[0].query(), "worker 0's apply was expected to still run"
        assert sh.stats["max_inflight"] >= 2
        torch.cuda.synchronize()
    finally:
        err = sh._error
        sh.stop()
        assert err is None, repr(err)
