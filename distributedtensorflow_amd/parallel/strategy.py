"""tf.distribute-style strategies, MI355X-native: one process per GPU, RCCL over xGMI.

BASELINE.json configs 1-5 name OneDevice / Mirrored / MultiWorkerMirrored /
ParameterServer strategies (none exist in the reference, which does TF1 between-graph PS
replication — ``run_mnist_distributed.py:104-161``).  Design:

* Every replica is its own OS process bound to one GPU (``LOCAL_RANK``); "in-graph" multi-GPU
  replication is deliberately not used — on MI355X one process per GPU with RCCL is the
  idiomatic (and fastest) layout.  ``MirroredStrategy`` over the 8 GPUs of a node and
  ``MultiWorkerMirroredStrategy`` across nodes are therefore the same engine; they differ only
  in how the cluster is discovered (env/torchrun vs ``TF_CONFIG``/``config.json``).
* Variables are created on the replica's device inside ``strategy.scope()`` (default device),
  then made identical by ONE broadcast of the optimizer's flat master buffer from rank 0.
* Gradients: the optimizer's flat fp32 gradient buffer is cut into contiguous buckets (sized for
  xGMI: a ring all-reduce is per-link bound, so few large buckets — default 64 MB — beat many
  small ones).  A post-accumulate hook counts each bucket's variables; the moment a bucket is
  complete its all-reduce is launched asynchronously on RCCL's stream while autograd keeps
  producing earlier-layer gradients on the compute stream (backward/communication overlap).
  The 1/N averaging is folded into the fused optimizer kernel's gradient scale.
"""
from __future__ import annotations

import contextlib
import functools
import os
import threading

import torch
import torch.distributed as dist

_tls = threading.local()
_default_strategy = None


class ReduceOp:
    SUM = "sum"
    MEAN = "mean"
    MAX = "max"
    MIN = "min"


def _torch_op(op):
    return {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.MEAN: dist.ReduceOp.SUM,
            ReduceOp.MAX: dist.ReduceOp.MAX, ReduceOp.MIN: dist.ReduceOp.MIN}[op]


def get_strategy():
    s = getattr(_tls, "strategy", None)
    if s is not None:
        return s
    global _default_strategy
    if _default_strategy is None:
        _default_strategy = _DefaultStrategy()
    return _default_strategy


def has_strategy():
    return getattr(_tls, "strategy", None) is not None


# ----------------------------------------------------------------------------- gradient reducers

class CommError(ConnectionError):
    """A collective or parameter-server transfer failed -- a peer process died or the transport
    broke.  Raised (from the transport's RuntimeError) only by this package's communication
    calls, so MonitoredTrainingSession can recover from exactly these and nothing else."""


def comm_call(fn):
    """Decorator for communication entry points: a transport RuntimeError (gloo's "Connection
    closed by peer", torch.distributed's DistError family) becomes :class:`CommError`; device
    faults (``torch.AcceleratorError``) stay what they are -- they are not recoverable by
    re-forming the cluster."""
    @functools.wraps(fn)
    def wrapper(*args, **kw):
        try:
            return fn(*args, **kw)
        except ConnectionError:
            raise
        except RuntimeError as e:
            if isinstance(e, getattr(torch, "AcceleratorError", ())):
                raise
            raise CommError(f"{type(e).__name__}: {e}") from e
    return wrapper


def force_reducer_default():
    """``DTF_FORCE_REDUCER=1``: build the communicating gradient reducer (and the process group)
    even when the world has ONE rank, so a ``torchrun --nproc-per-node 1`` run on the ``nccl``
    backend executes every hook, RCCL collective and ``finish()`` of the N > 1 path with the
    native ops' direct gradient writes (tests/test_forced_reducer_gpu.py)."""
    return os.environ.get("DTF_FORCE_REDUCER", "0") == "1"


class _NullReducer:
    def __init__(self, space=None):
        self.space = space

    def begin_step(self):
        pass

    def finish(self):
        pass

    def drain(self):
        """Complete any communication still in flight that writes the variables (the colocated
        parameter server's overlapped variable gather); a no-op for replicated strategies."""

    def gather_state(self, bufs):
        """Make flat optimizer-state buffers whole on every rank (sharded owners only)."""

    def grad_scale(self):
        return 1.0


class CommStats:
    """What the step's communication did, for the bench JSON and the overlap test.

    ``early`` / ``late``: buckets launched from the backward hooks (overlapped with autograd) vs
    launched only when ``finish()`` ran after backward.  ``exposed_ms``: time the compute stream
    waited for communication after backward (CUDA events around ``finish()``; host clock on
    CPU) -- the part of the all-reduce the overlap did not hide."""

    def __init__(self, n_buckets, bucket_bytes):
        self.n_buckets = n_buckets
        self.bucket_bytes = list(bucket_bytes)
        self.steps = 0
        self.early = 0
        self.late = 0
        self.last_early = 0
        self.timing = False
        self._events = []
        self._host_s = 0.0

    def reset_timing(self):
        self._events, self._host_s, self.steps, self.early, self.late = [], 0.0, 0, 0, 0

    def exposed_ms(self):
        """Total exposed communication time since ``reset_timing`` (synchronises)."""
        if self._events:
            torch.cuda.synchronize()
            return sum(a.elapsed_time(b) for a, b in self._events)
        return self._host_s * 1e3

    def as_dict(self):
        ms = self.exposed_ms()
        return {"buckets": self.n_buckets,
                "bucket_mb": [round(b / 2**20, 2) for b in self.bucket_bytes],
                "steps": self.steps, "early_launches": self.early, "late_launches": self.late,
                "exposed_ms_total": round(ms, 3),
                "exposed_ms_per_step": round(ms / max(self.steps, 1), 3)}


class BucketedAllReduce:
    """Overlapped bucketed all-reduce of a FlatSpace's gradient buffer.

    ``compress_bf16``: gradients travel as bf16 but are SUMMED in fp32 -- an all-to-all of bf16
    chunks (the reduce-scatter's data movement), a local fp32 sum of the W chunks each rank owns,
    then an all-gather of the bf16-rounded sums.  Each element is rounded twice (once per input,
    once per output: relative error <= 2^-8 of each term and of the sum, independent of the
    rank count), where an all-reduce run in bf16 would round at every one of the W-1 hops."""

    def __init__(self, space, group=None, bucket_bytes=64 << 20, first_bucket_bytes=4 << 20,
                 average=True, compress_bf16=False, overlap=True, comm=None):
        from .comm import C10dComm
        self.space = space
        self.group = group
        self.comm = comm if comm is not None else C10dComm(group)
        self.world = dist.get_world_size(group)
        self.average = average
        self.compress = compress_bf16
        # buckets over the decayed region in flat order (== reverse creation order), then one
        # bucket for the small non-decayed tail (BN gamma/beta, biases)
        ranges = []
        order, offs = space.order, space.offsets
        cur_start, cur_bytes, members = None, 0, []
        limit = first_bucket_bytes
        for i, (v, o) in enumerate(zip(order, offs)):
            if o >= space.decay_end and space.decay_end < space.numel:
                break
            if cur_start is None:
                cur_start = o
            members.append(i)
            end = offs[i + 1] if i + 1 < len(offs) else space.numel
            cur_bytes = (end - cur_start) * 4
            if cur_bytes >= limit:
                ranges.append((cur_start, end, members))
                cur_start, members, limit = None, [], bucket_bytes
        if members:
            ranges.append((cur_start, space.decay_end, members))
        tail = [i for i, o in enumerate(offs) if o >= space.decay_end and space.decay_end < space.numel]
        if tail:
            ranges.append((space.decay_end, space.numel, tail))
        self.buckets = ranges
        self.var_bucket = {}
        for b, (_, _, mem) in enumerate(ranges):
            for i in mem:
                self.var_bucket[i] = b
        self.pending = [0] * len(ranges)
        self.works = []
        self.launched = [False] * len(ranges)
        self.stats = CommStats(len(ranges), [(e - s) * 4 for s, e, _ in ranges])
        # collective issue order of the current / last completed step: every rank must issue
        # the same buckets in the same order (verify_bucket_agreement)
        self.launch_log = []
        self.last_order = ()
        # fault injection for the order check (tests): this rank defers every bucket to finish()
        # and issues them in reverse
        self._perturb = os.environ.get("DTF_DEBUG_PERTURB_BUCKET_ORDER", "") == \
            str(dist.get_rank(group))
        self._hooks = []
        for i, v in enumerate(order):
            if overlap:
                self._hooks.append(v.register_post_accumulate_grad_hook(self._make_hook(i)))
            # Ops that write their gradient straight into the flat buffer (ops/native.py
            # _direct_grad) return None for the variable, and autograd still runs the variable's
            # AccumulateGrad node -- once per backward, after every op that consumes the variable
            # (tied weights included) -- so the hook above already fires exactly once, after the
            # direct write.  Counting the ops' own readiness call as well launched buckets early
            # (caught by tests/test_distributed.py direct_grad_writes), so it is a no-op here.
            v._dtf_grad_ready = None

    def close(self, abort=False):
        """Detach the backward hooks (before a re-bucketed reducer replaces this one)."""
        self.works = []
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def _make_hook(self, i):
        def hook(_p):
            b = self.var_bucket[i]
            self.pending[b] -= 1
            if self.pending[b] == 0 and not self._perturb:
                self._launch(b)
        return hook

    @comm_call
    def _launch(self, b):
        if self.launched[b]:
            return
        self.launched[b] = True
        self.launch_log.append(b)
        s, e, _ = self.buckets[b]
        view = self.space.grad[s:e]
        if self.compress:
            W, L = self.world, e - s
            c = -(-L // W)
            send = torch.zeros(W * c, dtype=torch.bfloat16, device=view.device)
            send[:L].copy_(view)
            recv = torch.empty_like(send)
            w = dist.all_to_all_single(recv, send, group=self.group, async_op=True)
            self.works.append((w, view, (recv, c, L)))
        else:
            self.works.append((self.comm.all_reduce(view), None, None))

    def _finish_compressed(self, view, recv, c, L):
        W = self.world
        part = recv.view(W, c).float().sum(0).to(torch.bfloat16)   # fp32 sum of my chunk
        parts = [torch.empty_like(part) for _ in range(W)]
        return dist.all_gather(parts, part, group=self.group, async_op=True), view, parts, L

    def begin_step(self):
        self.pending = [len(m) for (_, _, m) in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []
        self.launch_log = []

    def plan(self):
        """The bucket plan as plain data: [(start, end, n_variables)] + the per-bucket owner
        pieces of a parameter-server reducer (reduce-scatter / all-gather chunk offsets)."""
        return {"buckets": [(s, e, len(m)) for s, e, m in self.buckets],
                "pieces": [list(p) for p in getattr(self, "pieces", [])]}

    def _timing_begin(self):
        st = self.stats
        if not st.timing:
            return None
        if self.space.grad.is_cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        import time
        return time.perf_counter()

    def _timing_end(self, t0):
        st = self.stats
        if t0 is None:
            return
        if isinstance(t0, torch.cuda.Event):
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            st._events.append((t0, ev))
        else:
            import time
            st._host_s += time.perf_counter() - t0

    @comm_call
    def finish(self):
        from .watchdog import check as _wd_check
        _wd_check()
        st = self.stats
        early = sum(self.launched)
        st.steps += 1
        st.early += early
        st.late += len(self.buckets) - early
        st.last_early = early
        t0 = self._timing_begin()
        # buckets whose variables received no gradient this step still have to be reduced
        for b in (range(len(self.buckets) - 1, -1, -1) if self._perturb
                  else range(len(self.buckets))):
            if not self.launched[b]:
                self._launch(b)
        self.last_order = tuple(self.launch_log)
        gathers = []
        for w, view, extra in self.works:
            w.wait()
            if extra is not None:
                gathers.append(self._finish_compressed(view, *extra))
        for w, view, parts, L in gathers:
            w.wait()
            view.copy_(torch.cat(parts)[:L])
        self.works = []
        self._timing_end(t0)

    def grad_scale(self):
        return 1.0 / self.world if self.average else 1.0

    def drain(self):
        pass

    def gather_state(self, bufs):
        pass


# ----------------------------------------------------------------------------- strategies

class Strategy:
    """Base: ``scope()``, ``run()``, ``reduce()``, ``experimental_distribute_dataset()``."""

    def __init__(self, device=None):
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._prev = None

    # -- replica topology
    @property
    def num_replicas_in_sync(self) -> int:
        return 1

    @property
    def replica_id(self) -> int:
        return 0

    @property
    def is_chief(self) -> bool:
        return self.replica_id == 0

    # -- context
    @contextlib.contextmanager
    def scope(self):
        prev = getattr(_tls, "strategy", None)
        _tls.strategy = self
        prev_dev = torch.get_default_device()
        torch.set_default_device(self.device)
        try:
            yield self
        finally:
            torch.set_default_device(prev_dev)
            _tls.strategy = prev

    def run(self, fn, args=(), kwargs=None):
        kwargs = kwargs or {}
        with self.scope():
            return fn(*args, **kwargs)

    def reduce(self, op, value, axis=None):
        if axis is not None:
            value = value.sum(axis) if op in (ReduceOp.SUM, ReduceOp.MEAN) else value
        return value

    def experimental_distribute_dataset(self, dataset):
        return dataset.shard(self.num_replicas_in_sync, self.replica_id) \
            if hasattr(dataset, "shard") and self.num_replicas_in_sync > 1 else dataset

    # -- variable sync hooks used by optimizers / checkpoints
    def make_gradient_reducer(self, space):
        return _NullReducer(space)

    def broadcast_space(self, space):
        pass

    def broadcast_tensors(self, tensors, src=0):
        pass

    def all_reduce_(self, t, op=ReduceOp.SUM):
        return t

    def barrier(self):
        pass

    @property
    def collective(self) -> bool:
        """True when the replicas are one synchronous collective world (every rank must enter
        checkpoint/state synchronisation together)."""
        return False

    def sync_after_restore(self, optimizer, global_step=None, restored=False):
        """After the chief restored a checkpoint: make every replica hold the chief's variables,
        optimizer slots, update count and global step (collective strategies only)."""


class _DefaultStrategy(Strategy):
    def __init__(self):
        super().__init__("cpu")

    @contextlib.contextmanager
    def scope(self):
        yield self


class OneDeviceStrategy(Strategy):
    """Single device, no communication.  ``OneDeviceStrategy("/cpu:0")`` is BASELINE config 1."""

    def __init__(self, device="/gpu:0"):
        super().__init__(_parse_device(device))


def _parse_device(d):
    if isinstance(d, torch.device):
        return d
    d = str(d).lower().strip("/")
    if d.startswith("cpu"):
        return torch.device("cpu")
    if d.startswith("gpu") or d.startswith("device:gpu"):
        idx = int(d.split(":")[-1]) if ":" in d else 0
        return torch.device("cuda", idx)
    return torch.device(d)


def _broadcast_training_state(active, optimizer, global_step=None, src=0, restored=False):
    """Rank ``src``'s master weights (+ compute shadow), optimizer slots, update count and global
    step to every rank: the state a restored chief hands to the other replicas.

    ``restored`` (meaningful on ``src``; broadcast so every rank takes the same branch): the chief
    holds a whole checkpoint.  When it does NOT, a parameter-server reducer's slot buffers are
    valid only on each chunk's owner, so they are gathered from the owners first -- broadcasting
    the chief's copy would overwrite every other owner's slots with stale values."""
    if not active or optimizer is None or optimizer.space is None:
        return
    optimizer.synchronize_variables()
    sp = optimizer.space
    flag = torch.tensor([1 if restored else 0], dtype=torch.int64, device=sp.device)
    dist.broadcast(flag, src)
    reducer = getattr(optimizer, "_reducer", None)
    if not int(flag[0]) and reducer is not None:
        reducer.gather_state(list(optimizer.state_tensors()))
    dist.broadcast(sp.master, src)
    for t in optimizer.state_tensors():
        dist.broadcast(t, src)
    meta = torch.tensor([optimizer.iterations,
                         global_step.value() if global_step is not None else 0],
                        dtype=torch.int64, device=sp.device)
    dist.broadcast(meta, src)
    optimizer.iterations = int(meta[0])
    if global_step is not None and hasattr(global_step, "assign"):
        global_step.assign(int(meta[1]))
    sp.refresh_shadow()


def _digest(obj):
    import hashlib
    return int.from_bytes(hashlib.sha1(repr(obj).encode()).digest()[:7], "little")


def verify_bucket_agreement(reducer, group=None):
    """Collective: every rank's bucket plan (bucket ranges, owner pieces) and the issue order of
    its last step's bucket collectives must be identical -- NCCL / RCCL match collectives by
    issue order, so a rank that issues them in another order sums the wrong buckets (or hangs).
    Returns the per-rank record [(n_buckets, plan_hash, order_hash)]; raises RuntimeError naming
    the ranks that disagree with rank 0."""
    plan = reducer.plan()
    mine = (len(plan["buckets"]), _digest(plan), _digest(tuple(reducer.last_order)))
    world = dist.get_world_size(group)
    dev = reducer.space.grad.device
    t = torch.tensor(mine, dtype=torch.int64, device=dev)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    recs = [tuple(int(v) for v in o.tolist()) for o in out]
    bad = [r for r, rec in enumerate(recs) if rec != recs[0]]
    if bad:
        raise RuntimeError(f"bucket plan / collective order differs from rank 0 on rank(s) {bad}: "
                           f"(buckets, plan hash, order hash) per rank = {recs}")
    return recs


_collective_watcher = None


def init_process_group_from_env(backend=None, timeout_s=None):
    """Initialise torch.distributed from torchrun-style env (RANK/WORLD_SIZE/MASTER_*).

    Under this package's launcher (``DTF_STORE_ADDR``: the launcher hosts the rendezvous store,
    cluster/rendezvous.py) the group is created for the current cluster EPOCH, and an epoch
    watcher tells the training session when a failed rank was restarted.

    Every world gets a fresh collective watchdog (parallel/watchdog.py): the communicators
    register their collectives with it, and the epoch bump is one of its failure probes, so a
    survivor blocked inside an RCCL kernel on a dead peer is released by an abort instead of
    waiting out the process-group timeout (``timeout_s``, default ``DTF_COMM_TIMEOUT_S`` = 300)."""
    import datetime
    global _collective_watcher
    if dist.is_initialized():
        return
    from . import comm as _comm, watchdog as _wd
    if timeout_s is None:
        timeout_s = _wd.default_timeout_s()
    _comm.reset_uid_index()
    wd = _wd.reset_watchdog()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    # RCCL watchdog: abort communicators whose collectives exceed the PG timeout instead of
    # hanging (a dead peer then surfaces as an error the session layer can recover from)
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    # ``timeout_s`` is the DTF watchdog's per-collective deadline.  The process group's own
    # timeout is strictly larger: under TORCH_NCCL_ASYNC_ERROR_HANDLING c10d's
    # watchdog tears the whole process down when it fires, so it must never win the race against
    # the controlled abort that turns a hung peer into a recoverable CommError.
    pg_timeout_s = pg_timeout_for(timeout_s)
    from ..cluster import rendezvous
    if rendezvous.store_address() is not None:
        store = rendezvous.connect(timeout_s)
        epoch = rendezvous.current_epoch(store)
        rendezvous.init_group(backend, rank, world, store, epoch, pg_timeout_s, **kw)
        if _collective_watcher is not None:
            _collective_watcher.stop()
        _collective_watcher = rendezvous.EpochWatcher(epoch).start()
        _collective_watcher.backend, _collective_watcher.timeout_s = backend, timeout_s
        _collective_watcher.store = store
        watcher = _collective_watcher
        wd.add_probe(lambda: (f"cluster epoch moved past {watcher.epoch}: a peer was restarted"
                              if watcher.changed else None))
        return
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
        # torchrun: its agent already hosts the store and ran the rendezvous
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=pg_timeout_s), **kw)
        return
    # the rendezvous waits for every rank's process to START (imports, device init): bound it
    # separately from the collective deadline, which may be seconds (DTF_COMM_TIMEOUT_S)
    rdv_s = max(float(timeout_s), float(os.environ.get("DTF_RENDEZVOUS_TIMEOUT_S", "300") or 300))
    store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                          rank == 0, timeout=datetime.timedelta(seconds=rdv_s))
    dist.init_process_group(backend, store=store, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=pg_timeout_s), **kw)


def pg_timeout_for(deadline_s):
    """Process-group timeout for a watchdog deadline: ``max(2 x deadline, deadline + 60 s)``."""
    d = float(deadline_s)
    return max(2.0 * d, d + 60.0)


def collective_cluster_changed():
    """True once a peer was restarted (epoch bump) or the collective watchdog tripped (a
    collective missed its deadline or the communicator reported an error)."""
    from .watchdog import _watchdog as wd
    if wd is not None and wd.failed is not None:
        return True
    return _collective_watcher is not None and _collective_watcher.changed


def rejoin_collective(timeout_s=120.0):
    """A rank of the collective world died: leave the broken group, wait until the launcher has
    restarted it (epoch bump; bounded) and join the new epoch's group with every other rank."""
    from ..cluster import rendezvous
    w = _collective_watcher
    if w is None:
        raise RuntimeError("collective recovery needs the launcher's rendezvous store "
                           "(DTF_STORE_ADDR)")
    rendezvous.leave_group()
    rendezvous.wait_for_epoch_after(w.store, w.epoch, timeout_s)
    init_process_group_from_env(w.backend, w.timeout_s)
    return _collective_watcher.epoch


class MirroredStrategy(Strategy):
    """Synchronous data parallelism: replicated variables, all-reduced gradients (RCCL).

    One process per GPU; ``devices`` (TF signature) is accepted for API compatibility but the
    replica set is the torch.distributed world of this node.  With ``WORLD_SIZE`` unset it
    runs single-replica on ``cuda:LOCAL_RANK``.
    """

    def __init__(self, devices=None, cross_device_ops=None, bucket_mb=64, first_bucket_mb=4,
                 compress_bf16=False, backend=None, overlap=True, force_reducer=None, comm=None):
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            dev = torch.device("cuda", local)
        else:
            dev = torch.device("cpu")
        super().__init__(dev)
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.first_bucket_bytes = int(first_bucket_mb * (1 << 20))
        self.compress_bf16 = compress_bf16
        self.overlap = overlap
        self.comm_kind = comm             # "c10d" / "rccl" / None (DTF_COMM, default c10d)
        self._comm = None
        self.force_reducer = force_reducer_default() if force_reducer is None else force_reducer
        if int(os.environ.get("WORLD_SIZE", "1")) > 1 or self.force_reducer:
            init_process_group_from_env(backend)
        self._dist = dist.is_initialized() and (dist.get_world_size() > 1 or self.force_reducer)

    @property
    def num_replicas_in_sync(self):
        return dist.get_world_size() if self._dist else 1

    @property
    def replica_id(self):
        return dist.get_rank() if self._dist else 0

    def communicator(self):
        """The gradient communicator of this world (created once; see parallel/comm.py)."""
        if self._comm is None:
            from .comm import make_comm
            self._comm = make_comm(self.comm_kind, None, self.device)
        return self._comm

    def make_gradient_reducer(self, space):
        if not self._dist:
            return _NullReducer(space)
        return BucketedAllReduce(space, None, self.bucket_bytes, self.first_bucket_bytes,
                                 compress_bf16=self.compress_bf16, overlap=self.overlap,
                                 comm=None if self.compress_bf16 else self.communicator())

    def broadcast_space(self, space):
        if self._dist:
            dist.broadcast(space.master, 0)
            space.refresh_shadow()

    def broadcast_tensors(self, tensors, src=0):
        if self._dist:
            for t in tensors:
                dist.broadcast(t, src)

    @property
    def collective(self):
        return self._dist

    def sync_after_restore(self, optimizer, global_step=None, restored=False):
        _broadcast_training_state(self._dist, optimizer, global_step, restored=restored)

    def cluster_changed(self):
        return collective_cluster_changed()

    def recover_cluster(self, optimizer=None):
        """A replica died and the launcher restarted it: re-form the world in the new epoch and
        rebuild the gradient reducer on the new process group (the caller restores the latest
        checkpoint on the chief and calls :meth:`sync_after_restore`)."""
        # the cached communicator belongs to the old world (it includes the dead peer): abort
        # it BEFORE leaving, so nothing of it survives into the new epoch (the PS strategy does
        # the same, ps_strategy.recover_cluster)
        if optimizer is not None and hasattr(getattr(optimizer, "_reducer", None), "close"):
            optimizer._reducer.close(abort=True)
        if self._comm is not None:
            try:
                self._comm.close(abort=True)
            except Exception:
                pass
            self._comm = None
        epoch = rejoin_collective()
        self._dist = dist.is_initialized() and (dist.get_world_size() > 1 or self.force_reducer)
        if optimizer is not None and optimizer.space is not None:
            optimizer._reducer = self.make_gradient_reducer(optimizer.space)
            # the restarted replica's Optimizer.build broadcast, mirrored (the collective
            # sequence must be the same on every rank)
            self.broadcast_space(optimizer.space)
        return epoch

    def reduce(self, op, value, axis=None):
        value = super().reduce(op, value, axis)
        if not self._dist:
            return value
        t = value.detach().clone() if isinstance(value, torch.Tensor) else torch.tensor(
            float(value), device=self.device)
        dist.all_reduce(t, _torch_op(op))
        if op == ReduceOp.MEAN:
            t /= self.num_replicas_in_sync
        return t

    def all_reduce_(self, t, op=ReduceOp.SUM):
        if self._dist:
            dist.all_reduce(t, _torch_op(op))
            if op == ReduceOp.MEAN:
                t /= self.num_replicas_in_sync
        return t

    def barrier(self):
        if self._dist:
            dist.barrier()


class MultiWorkerMirroredStrategy(MirroredStrategy):
    """Same engine as MirroredStrategy; cluster from ``TF_CONFIG`` / config.json when torchrun
    env is absent (one process per GPU on every worker host)."""

    def __init__(self, cluster_resolver=None, communication=None, **kw):
        if "WORLD_SIZE" not in os.environ and (cluster_resolver is not None or
                                               "TF_CONFIG" in os.environ):
            from ..cluster import resolver as _res
            _res.export_torch_env(cluster_resolver)
        super().__init__(**kw)
