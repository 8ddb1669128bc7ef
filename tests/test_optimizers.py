"""TF1-exact optimizer math (SURVEY.md §4 'unit tests for optimizer math'): every optimizer's
flat-buffer update is compared with a per-tensor numpy transcription of the TF kernels
(training_ops.cc ApplyAdam / ApplyAdagrad / ApplyMomentum) over several steps, on CPU; the GPU
test runs the fused HIP update kernels against the same oracle."""
import math

import numpy as np
import pytest
import torch

import distributedtensorflow_amd as dtf
from distributedtensorflow_amd.optimizers import (AdagradOptimizer, AdamOptimizer,
                                                  GradientDescentOptimizer, LAMBOptimizer,
                                                  MomentumOptimizer)
from distributedtensorflow_amd.optimizers.optimizers import (clip_by_global_norm_, cosine_decay,
                                                             piecewise_constant, polynomial_decay)
from distributedtensorflow_amd.parallel import OneDeviceStrategy


def _params(device, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(7, 5), (5,), (3, 3, 2, 4), (130,)]
    names = ["dense/kernel", "dense/bias", "conv2d/kernel", "bn/gamma"]
    ps = []
    for s, n in zip(shapes, names):
        p = torch.nn.Parameter(torch.randn(s, generator=g, device="cpu").to(device))
        p._dtf_name = n
        ps.append(p)
    return ps


def _grads(ps, step):
    g = torch.Generator().manual_seed(100 + step)
    return [torch.randn(p.shape, generator=g, device="cpu") for p in ps]


def _run(opt, device, steps=4):
    ps = _params(device)
    ref = [p.detach().cpu().double().numpy().copy() for p in ps]
    with OneDeviceStrategy(device).scope():
        opt.build(ps)
        for t in range(steps):
            gs = _grads(ps, t)
            opt.space.zero_grad()
            for p, g in zip(ps, gs):
                p.grad.copy_(g.to(device))
            opt.apply_gradients()
            yield t, [p.detach().cpu().double().numpy() for p in ps], \
                [g.double().numpy() for g in gs], ref


def _decay(name):
    return not ("bias" in name or "gamma" in name)


def check(opt_factory, oracle, device="cpu", rtol=1e-5, atol=1e-6, steps=4):
    opt = opt_factory()
    state = None
    for t, got, gs, ref in _run(opt, device, steps):
        if state is None:
            state = [oracle.init(r) for r in ref]
            cur = [r.copy() for r in ref]
        names = ["dense/kernel", "dense/bias", "conv2d/kernel", "bn/gamma"]
        for i, (g, n) in enumerate(zip(gs, names)):
            cur[i] = oracle.step(cur[i], g, state[i], t + 1, _decay(n))
        for a, b in zip(got, cur):
            np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


class Adam:
    def __init__(self, lr, b1=0.9, b2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps

    def init(self, p):
        return {"m": np.zeros_like(p), "v": np.zeros_like(p)}

    def step(self, p, g, s, t, dec):
        lr_t = self.lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
        s["m"] = self.b1 * s["m"] + (1 - self.b1) * g
        s["v"] = self.b2 * s["v"] + (1 - self.b2) * g * g
        return p - lr_t * s["m"] / (np.sqrt(s["v"]) + self.eps)


class Adagrad:
    def __init__(self, lr, acc0=0.1):
        self.lr, self.acc0 = lr, acc0

    def init(self, p):
        return {"a": np.full_like(p, self.acc0)}

    def step(self, p, g, s, t, dec):
        s["a"] = s["a"] + g * g
        return p - self.lr * g / np.sqrt(s["a"])


class Momentum:
    def __init__(self, lr, mu, nesterov=False, wd=0.0):
        self.lr, self.mu, self.nesterov, self.wd = lr, mu, nesterov, wd

    def init(self, p):
        return {"a": np.zeros_like(p)}

    def step(self, p, g, s, t, dec):
        g = g + (self.wd * p if dec else 0.0)
        s["a"] = self.mu * s["a"] + g
        upd = g + self.mu * s["a"] if self.nesterov else s["a"]
        return p - self.lr * upd


class Lamb:
    def __init__(self, lr, wd, b1=0.9, b2=0.999, eps=1e-6):
        self.lr, self.wd, self.b1, self.b2, self.eps = lr, wd, b1, b2, eps

    def init(self, p):
        return {"m": np.zeros_like(p), "v": np.zeros_like(p)}

    def step(self, p, g, s, t, dec):
        s["m"] = self.b1 * s["m"] + (1 - self.b1) * g
        s["v"] = self.b2 * s["v"] + (1 - self.b2) * g * g
        u = (s["m"] / (1 - self.b1 ** t)) / (np.sqrt(s["v"] / (1 - self.b2 ** t)) + self.eps)
        u = u + (self.wd * p if dec else 0.0)
        pn, un = np.linalg.norm(p), np.linalg.norm(u)
        r = pn / un if pn > 0 and un > 0 else 1.0
        return p - self.lr * r * u


CASES = [
    ("adam", lambda: AdamOptimizer(5e-4), Adam(5e-4)),
    ("adam_big_lr", lambda: AdamOptimizer(0.01, 0.8, 0.99, 1e-6), Adam(0.01, 0.8, 0.99, 1e-6)),
    ("adagrad", lambda: AdagradOptimizer(0.01), Adagrad(0.01)),
    ("sgd", lambda: GradientDescentOptimizer(0.1), Momentum(0.1, 0.0)),
    ("momentum", lambda: MomentumOptimizer(0.1, 0.9), Momentum(0.1, 0.9)),
    ("nesterov", lambda: MomentumOptimizer(0.05, 0.9, use_nesterov=True),
     Momentum(0.05, 0.9, True)),
    ("momentum_wd", lambda: MomentumOptimizer(0.1, 0.9, weight_decay=1e-4),
     Momentum(0.1, 0.9, wd=1e-4)),
    ("lamb", lambda: LAMBOptimizer(1e-3, weight_decay=0.01), Lamb(1e-3, 0.01)),
]


@pytest.mark.parametrize("name,factory,oracle", CASES, ids=[c[0] for c in CASES])
def test_optimizer_matches_tf_math_cpu(name, factory, oracle):
    check(factory, oracle, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("name,factory,oracle", CASES, ids=[c[0] for c in CASES])
def test_optimizer_kernels_gpu(name, factory, oracle):
    check(factory, oracle, "cuda", rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
def test_optimizer_shadow_and_nonfinite_gpu():
    ps = _params("cuda")
    opt = MomentumOptimizer(0.1, 0.9)
    with OneDeviceStrategy("cuda").scope():
        opt.build(ps)
        for p in ps:
            p.grad.fill_(1.0)
        opt.apply_gradients()
        torch.cuda.synchronize()
        for p in ps:
            assert p._dtf_shadow.dtype == torch.bfloat16
            torch.testing.assert_close(p._dtf_shadow.float(), p.detach().bfloat16().float())
        assert not opt.nonfinite_flag()
        ps[0].grad[0, 0] = float("nan")
        opt.apply_gradients()
        assert opt.nonfinite_flag()


def test_flat_space_layout():
    ps = _params("cpu")
    opt = GradientDescentOptimizer(0.1)
    with OneDeviceStrategy("cpu").scope():
        sp = opt.build(ps)
    # reverse creation order, decayed first; every view 64-element aligned
    names = [p._dtf_name for p in sp.order]
    assert names == ["conv2d/kernel", "dense/kernel", "bn/gamma", "dense/bias"]
    assert all(o % 64 == 0 for o in sp.offsets)
    assert sp.regions()[0][2] and not sp.regions()[1][2]
    for p in ps:
        assert p.data.data_ptr() == sp.view_of(sp.master, p).data_ptr()
        assert p.grad.data_ptr() == sp.view_of(sp.grad, p).data_ptr()


def test_minimize_and_global_step():
    torch.manual_seed(0)
    x = torch.randn(64, 4)
    w_true = torch.tensor([[1.0], [-2.0], [0.5], [3.0]])
    y = x @ w_true
    w = torch.nn.Parameter(torch.zeros(4, 1))
    w._dtf_name = "w"
    with OneDeviceStrategy("cpu").scope():
        gstep = dtf.train.get_or_create_global_step()
        opt = AdamOptimizer(0.1)
        for _ in range(300):
            loss = ((x @ w - y) ** 2).mean()
            opt.minimize(loss, global_step=gstep)
    assert int(gstep) == 300
    torch.testing.assert_close(w.detach(), w_true, atol=2e-2, rtol=0)


def test_range_restricted_apply():
    """Colocated parameter-server shards update only the variables in their range."""
    ps = _params("cpu")
    opt = AdamOptimizer(0.1)
    with OneDeviceStrategy("cpu").scope():
        sp = opt.build(ps)
    before = sp.master.clone()
    sp.grad.fill_(1.0)
    opt.iterations = 1
    lo, hi = sp.offsets[1], sp.offsets[2]
    opt._apply(1.0, (lo, hi))
    changed = (sp.master != before).nonzero().flatten()
    assert changed.min() >= lo and changed.max() < hi


def test_lamb_range_restricted_apply():
    ps = _params("cpu")
    opt = LAMBOptimizer(0.1)
    with OneDeviceStrategy("cpu").scope():
        sp = opt.build(ps)
    before = sp.master.clone()
    sp.grad.fill_(1.0)
    opt.iterations = 1
    lo, hi = sp.offsets[1], sp.offsets[3]
    opt._apply(1.0, (lo, hi))
    changed = (sp.master != before).nonzero().flatten()
    assert changed.min() >= lo and changed.max() < hi


def test_clip_by_global_norm():
    ps = _params("cpu")
    opt = GradientDescentOptimizer(0.1)
    with OneDeviceStrategy("cpu").scope():
        sp = opt.build(ps)
    sp.grad.normal_()
    n0 = sp.grad.norm().item()
    norm = clip_by_global_norm_(sp, 1.0)
    assert abs(norm.item() - n0) < 1e-4
    assert abs(sp.grad.norm().item() - 1.0) < 1e-4


def test_schedules():
    f = polynomial_decay(1.0, 100, end_lr=0.0, warmup_steps=10)
    assert f(0) == pytest.approx(0.1) and f(9) == pytest.approx(1.0)
    assert f(50) == pytest.approx(0.5) and f(1000) == 0.0
    g = piecewise_constant([10, 20], [1.0, 0.1, 0.01])
    assert (g(0), g(10), g(25)) == (1.0, 0.1, 0.01)
    c = cosine_decay(1.0, 100)
    assert c(0) == pytest.approx(1.0) and c(100) == pytest.approx(0.0, abs=1e-12)


def test_optimizer_config_roundtrip():
    for opt in [AdamOptimizer(0.01), AdagradOptimizer(0.01), MomentumOptimizer(0.1, 0.9),
                GradientDescentOptimizer(0.5), LAMBOptimizer(1e-3)]:
        cfg = dict(opt.get_config())
        kind = cfg.pop("type")
        clone = type(opt)(**cfg)
        assert clone.get_config()["type"] == kind


def test_sync_replicas_backup_workers_need_between_graph_ps():
    """Collective strategies aggregate every replica each step; asking them for backup workers
    (replicas_to_aggregate < replicas) must raise instead of silently ignoring it."""
    from distributedtensorflow_amd.optimizers import AdamOptimizer
    from distributedtensorflow_amd.optimizers.sync_replicas import SyncReplicasOptimizer
    from distributedtensorflow_amd.parallel.strategy import Strategy

    class TwoReplicas(Strategy):
        num_replicas_in_sync = 2

    with TwoReplicas("cpu").scope():
        SyncReplicasOptimizer(AdamOptimizer(0.1), replicas_to_aggregate=2)     # all replicas: ok
        with pytest.raises(ValueError, match="backup workers"):
            SyncReplicasOptimizer(AdamOptimizer(0.1), replicas_to_aggregate=1,
                                  total_num_replicas=2)


def test_graphed_train_step_needs_gpu():
    """HIP-graph capture of a training step (train/graphed.py) is GPU-only; on a CPU host it
    refuses up front instead of failing inside torch.cuda.graph."""
    import torch as _t
    from distributedtensorflow_amd.train import GraphedTrainStep
    if _t.cuda.is_available():
        pytest.skip("CPU-only check")
    with pytest.raises(RuntimeError, match="GPU"):
        GraphedTrainStep(lambda x: x, None, [_t.zeros(1)])
