"""The pipelined push/pull state machine of the between-graph PS (``ps_strategy._RemotePSReducer``)
on the CPU: the same code the GPU runs, with ``_Streams``' synchronous CPU stand-ins for the HIP
side stream and its events (this path had no CPU coverage).

Covered: a step pushes every bucket from the backward hooks and posts on the generation's comm
thread; the next forward's fence receives the answer and pulls; ``reset_pipeline`` (recovery)
cancels a push whose answer never comes within one 200 ms wait slice, retires the comm thread,
removes the module pre-hook and the op fence; the next generation gets a fresh comm thread that a
stuck job of the old one cannot delay; gradients modified in place after backward (clipping) are
copied again before the post."""
import threading
import time

import pytest
import torch

from distributedtensorflow_amd import ops
from distributedtensorflow_amd.optimizers.base import FlatSpace
from distributedtensorflow_amd.parallel import ps_strategy
from distributedtensorflow_amd.parallel.ps_strategy import _RemotePSReducer


class FakeLink:
    """A PSLink stand-in: one mailbox = the whole flat buffer, answers when ``release``d."""

    def __init__(self, space, auto_answer=True):
        self.mail = torch.zeros(space.numel)
        self.owner = torch.zeros(space.numel)
        self.timeout_ms = 3000
        self.posted = []
        self.auto = auto_answer
        self._answer = threading.Event()
        self.step = 0
        self.cancelled_waits = 0

    def copy_grads(self, space, lo=None, hi=None):
        lo, hi = lo or 0, hi if hi is not None else space.numel
        self.mail[lo:hi].copy_(space.grad[lo:hi])

    def post(self, step):
        self.posted.append((step, self.mail.clone()))
        if self.auto:
            self._answer.set()

    def wait(self, cancelled=None):
        while not self._answer.wait(0.05):
            if cancelled is not None and cancelled():
                self.cancelled_waits += 1
                raise ConnectionError("cancelled")
        self._answer.clear()
        self.step += 1
        self.owner.add_(1.0)              # the owner "applied": every variable moves by +1
        return self.step

    def pull(self, space, lo=None, hi=None):
        lo, hi = lo or 0, hi if hi is not None else space.numel
        space.master[lo:hi].copy_(self.owner[lo:hi])

    @property
    def global_step(self):
        return self.step


class FakeClient:
    def __init__(self, links):
        self.links = links
        self.global_step = 0


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(8, 16)
        self.b = torch.nn.Linear(16, 4)

    def forward(self, x):
        return self.b(torch.relu(self.a(x)))


def _setup(auto=True, bucket_bytes=256):
    torch.manual_seed(0)
    net = Net()
    space = FlatSpace(list(net.parameters()))
    link = FakeLink(space, auto)
    client = FakeClient([link])
    red = _RemotePSReducer(space, client, bucket_bytes=bucket_bytes)
    return net, space, link, client, red


def _step(net, space, red, modify=None):
    space.zero_grad()
    red.begin_step()
    net(torch.randn(3, 8)).square().sum().backward()
    red.finish()
    if modify is not None:
        modify(net)
    return red.apply_remote(None)


@pytest.fixture(autouse=True)
def _clean_fence():
    yield
    ops.set_param_fence(None)


def test_pipelined_step_pushes_posts_and_pulls_at_next_forward():
    net, space, link, client, red = _setup()
    assert len(red.buckets) > 1
    step = _step(net, space, red)
    assert red.pipelined() and step == 1
    assert red._pre_hook is not None and ops._PARAM_FENCE is not None
    assert red._job._done.wait(2.0)          # the comm thread posted and got the answer
    # the first step's buckets are pushed at apply time (the mode is decided then); the mailbox
    # holds exactly the gradients
    assert link.posted[0][0] == 0 and torch.equal(link.posted[0][1], space.grad)
    # the next forward's module fence takes the answer and pulls every bucket
    net(torch.randn(2, 8))
    assert client.global_step == 1 and ops._PARAM_FENCE is None
    assert torch.equal(space.master, torch.ones(space.numel))
    # steady state: the hooks push during backward, before apply_remote
    pushed = []
    orig = link.copy_grads
    link.copy_grads = lambda sp, lo=None, hi=None: (pushed.append((lo, hi)), orig(sp, lo, hi))
    _step(net, space, red)
    assert len(pushed) == len(red.buckets) and red.repushed == 0
    red.drain()
    assert client.global_step == 2


def test_reset_cancels_a_stalled_push_and_starts_a_new_generation():
    net, space, link, client, red = _setup(auto=False)
    _step(net, space, red)
    job, comm, hook = red._job, red._comm, red._pre_hook
    assert job is not None and hook is not None
    time.sleep(0.2)                          # the comm thread is now inside link.wait
    t0 = time.perf_counter()
    red.reset_pipeline(join_s=3.0)
    assert time.perf_counter() - t0 < 1.0, "cancel must end the wait within a slice"
    assert job._done.is_set() and isinstance(job._error, ConnectionError)
    assert link.cancelled_waits == 1
    assert red._job is None and red._pipe is None and red._pre_hook is None
    assert red._comm is None and red.generation == 1 and ops._PARAM_FENCE is None
    assert not any(red.launched)         # the retried step pushes every bucket to the new shard
    comm.t.join(2.0)
    assert not comm.t.is_alive(), "the old generation's comm thread must be retired"
    # generation 1: a new link answers; a fresh comm thread serves it
    link2 = FakeLink(space, auto_answer=True)
    client.links = [link2]
    _step(net, space, red)
    assert red._comm is not None and red._comm is not comm
    red.drain()
    assert client.global_step == 1 and len(link2.posted) == 1
    assert torch.equal(link2.posted[0][1], space.grad)


def test_stuck_old_generation_cannot_delay_the_new_one():
    """A job of the old generation that ignores the cancel (its link never answers and never
    checks the flag) holds only ITS comm thread: the next generation's push completes."""
    net, space, link, client, red = _setup(auto=False)
    link.wait = lambda cancelled=None: time.sleep(30)      # ignores cancellation
    _step(net, space, red)
    time.sleep(0.1)
    t0 = time.perf_counter()
    red.reset_pipeline(join_s=0.3)
    assert time.perf_counter() - t0 < 1.5
    link2 = FakeLink(space, auto_answer=True)
    client.links = [link2]
    _step(net, space, red)
    t0 = time.perf_counter()
    red.drain()
    assert time.perf_counter() - t0 < 2.0 and client.global_step == 1


def test_no_answer_within_deadline_raises_timeout_naming_the_step():
    net, space, link, client, red = _setup(auto=False)
    link.timeout_ms = 0                       # deadline = links' + 10 s; shorten it for the test
    _step(net, space, red)
    red._job.deadline_s = 0.3
    with pytest.raises(TimeoutError, match="global step 0"):
        red.drain()
    red.reset_pipeline(join_s=1.0)


def test_gradients_clipped_after_backward_are_pushed_as_clipped():
    net, space, link, client, red = _setup()
    _step(net, space, red)
    red.drain()

    def clip(n):
        with torch.no_grad():
            for p in n.parameters():
                p.grad.mul_(0.5)
    _step(net, space, red, modify=clip)
    assert red.repushed == 1 and red._job._done.wait(2.0)
    assert torch.equal(link.posted[-1][1], space.grad)      # the halved gradients were posted
    red.drain()
    _step(net, space, red)                                  # unmodified: no extra copies
    assert red.repushed == 1
    red.drain()


def test_close_removes_every_hook():
    net, space, link, client, red = _setup()
    _step(net, space, red)
    red.close()
    assert red._hooks == [] and red._pre_hook is None and ops._PARAM_FENCE is None
    assert all(getattr(v, "_dtf_gbucket", None) is None for v in space.order)


def test_pipeline_env_switch(monkeypatch):
    monkeypatch.setenv("DTF_PS_PIPELINE", "0")
    net, space, link, client, red = _setup()
    assert not ps_strategy.pipeline_enabled(space.device)
    monkeypatch.setenv("DTF_PS_PIPELINE", "1")
    assert ps_strategy.pipeline_enabled(space.device)
