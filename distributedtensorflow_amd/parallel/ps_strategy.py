"""ParameterServerStrategy (BASELINE.json config 4; reference R6/R13/T6/T7).

Two deployments of the same semantics — variables are OWNED by parameter-server shards, workers
compute gradients, owners apply the optimizer, workers read back the new values:

* **between-graph** (``ParameterServerStrategy(server=Server(...))``): the reference's layout —
  separate ``ps`` tasks run :class:`~.ps_service.ParameterServerService` (``server.join()``);
  workers pull/push over the gloo world (async Hogwild by default, ``sync=True`` =
  SyncReplicasOptimizer aggregation with stale-gradient drop).
* **colocated, synchronous, on RCCL** (no ``server``; one process per GPU under torchrun): the
  PS shards are hosted by the GPU ranks themselves (``num_ps`` owners; 1 = "1 PS + N workers",
  default = every rank owns an equal chunk of every gradient bucket).  Per step: as soon as a
  gradient bucket is complete during backward it is reduce-scattered to its owners over xGMI
  (``reduce`` per owner piece when num_ps < world), overlapped with the rest of backward; after
  backward each owner runs the fused optimizer on exactly its chunks and the updated masters
  are all-gathered (``broadcast`` from the owner when num_ps < world) bucket by bucket,
  overlapped with the next forward (see :class:`_ColocatedPSReducer`).
"""
from __future__ import annotations

import os
import threading
import time

import torch
import torch.distributed as dist

from .strategy import (BucketedAllReduce, MirroredStrategy, Strategy, _broadcast_training_state,
                       _NullReducer, collective_cluster_changed, comm_call,
                       force_reducer_default, init_process_group_from_env, rejoin_collective)



class _RemotePSReducer(_NullReducer):
    """Between-graph: push the gradients at step end; the reply carries the updated variables
    (so the NEXT forward pass reads fresh values — TF's read-at-step-start semantics).

    **Pipelined async push/pull** (device data plane -- HBM shard over hipIpc, or a /dev/shm
    shard for CPU tasks --, async mode; ``DTF_PS_PIPELINE=0`` turns it off).  The serial form --
    compute, full device sync, copy into the mailbox, post, wait for the owner's answer, copy
    the variables back -- leaves the GPU idle while the host waits, and at 8 workers over xGMI
    the 2 x 102 MB of ResNet-50 traffic per step becomes real time.  Pipelined, nothing on the
    worker's compute stream waits for the host:

    * **push from the backward hooks**: the gradient buffer is cut into buckets (as for the
      all-reduce); the moment a bucket's last gradient lands, its mailbox copies are enqueued on
      a side stream behind an event of the compute stream, overlapped with the rest of backward;
    * **post / answer on a comm thread**: ``apply_remote`` records the push-complete event and
      hands (event, step) to this generation's comm thread, which waits for it, posts to every
      owner and waits for the answers -- the main thread goes straight on to issue the next step;
    * **pull fenced per bucket into the next forward**: the first op of the next forward that
      reads a bucket's variables (``ops`` parameter fence + a module forward pre-hook) waits for
      the answer (host, bounded), enqueues every bucket's pull copy on the side stream in
      FORWARD order with one event each, and makes the compute stream wait only for ITS bucket:
      the late layers' variables keep streaming in while the early layers compute.

    The stream/event operations go through :class:`_Streams`: HIP streams and events on a GPU,
    an ordered-synchronous stand-in on the CPU, so the same state machine (including recovery,
    :meth:`reset_pipeline`) runs -- and is tested -- on CPU tasks with the /dev/shm plane.

    **Generations.**  A recovery (a PS died; the cluster re-forms) calls :meth:`reset_pipeline`
    BEFORE leaving the old process group: the push in flight is cancelled (its answer wait
    checks the flag every 200 ms slice) and joined with a deadline, the side stream is drained,
    the comm thread of the old generation is retired (a new one serves the next generation, so
    a push stuck on the old control block can never delay a new one) and the module pre-hook
    is removed (one hook per live generation, never one per recovery).

    **Gradients modified after backward** (clipping between ``compute_gradients`` and
    ``apply_gradients``): the gradient buffer's version counter is recorded when the last bucket
    was pushed; ``apply_remote`` re-copies every bucket when it moved, so the owner always gets
    the gradients as they are at apply time, like the serial data plane.

    Semantics are the reference's (``run_mnist_distributed.py:107-116,150,161``): a worker's
    next forward reads the variables after its own update was applied (plus whatever other
    workers applied meanwhile, Hogwild).  The global step ``apply_remote`` reports is the one
    the push in flight will at least produce: exact with one worker, a lower bound with more
    (the serial form's answer also counts other workers' pushes applied meanwhile), so with N
    workers ``StopAtStepHook`` may let a worker run one step more than the serial plane would;
    ``drain()`` completes the push and makes the step exact."""

    applies_update = True

    def __init__(self, space, client, sync=False, bucket_bytes=32 << 20):
        super().__init__(space)
        self.client = client
        self.sync = sync
        self._pipe = None            # decided at the first step (the links exist after register)
        self.buckets = _bucket_plan(space, bucket_bytes)
        self.var_bucket = {i: b for b, (_, _, mem) in enumerate(self.buckets) for i in mem}
        self.pending = [0] * len(self.buckets)
        self.launched = [False] * len(self.buckets)
        self._hooks = [v.register_post_accumulate_grad_hook(self._make_hook(i))
                       for i, v in enumerate(space.order)]
        for b, (_, _, mem) in enumerate(self.buckets):
            for i in mem:
                space.order[i]._dtf_gbucket = b
        self._pre_hook = None
        self._streams = None
        self._comm = None            # this generation's comm thread
        self._job = None             # the push in flight: a _PushJob
        self._pull_events = None     # per bucket, after the answer: event of its pull copy
        self._fenced = 0
        self._pushed_version = None  # space.grad._version when the last bucket was pushed
        self.generation = 0
        self.timing = {"fence_ms": [], "answer_ms": []}
        self.repushed = 0            # steps whose gradients changed after backward pushed them

    # -- mode
    def pipelined(self):
        if self._pipe is None:
            c = self.client
            self._pipe = bool(c.links) and not self.sync and pipeline_enabled(self.space.device)
            if self._pipe:
                self._streams = _Streams(self.space.device)
                self._comm = _CommThread(f"dtf-ps-push-g{self.generation}")
                if self._pre_hook is None:
                    from torch.nn.modules.module import register_module_forward_pre_hook
                    self._pre_hook = register_module_forward_pre_hook(self._module_fence)
        return self._pipe

    # -- push (backward)
    def begin_step(self):
        if self._pipe:
            self.drain()
            self.pending = [len(m) for (_, _, m) in self.buckets]
            self.launched = [False] * len(self.buckets)
            self._pushed_version = None

    def _make_hook(self, i):
        def hook(_p):
            if not self._pipe:
                return
            b = self.var_bucket[i]
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self._push_bucket(b)
        return hook

    def _push_bucket(self, b, force=False):
        if self.launched[b] and not force:
            return
        self.launched[b] = True
        s, e, _ = self.buckets[b]
        st = self._streams
        st.side_waits_compute()
        with st.side():
            for link in self.client.links:
                link.copy_grads(self.space, s, e)
        if all(self.launched):
            self._pushed_version = self.space.grad._version

    def finish(self):
        if self._pipe:
            for b in range(len(self.buckets)):
                if not self.launched[b]:
                    self._push_bucket(b)

    @comm_call
    def apply_remote(self, optimizer):
        if not self.pipelined():
            params = self.space.order
            return self.client.push([p.grad for p in params], pull=True)
        # buckets the backward hooks did not push (the first pipelined step, decided only now;
        # variables without a gradient this step)
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._push_bucket(b)
        if self._pushed_version is not None and self.space.grad._version != self._pushed_version:
            # the gradients were modified in place after backward pushed them (clipping, ...):
            # the mailbox must hold what the serial plane would send -- copy every bucket again
            self.repushed += 1
            for b in range(len(self.buckets)):
                self._push_bucket(b, force=True)
        st = self._streams
        ev = st.record()
        # the next step's zero_grad (compute stream) must not overwrite the gradient buffer
        # under the side stream's mailbox copies
        st.compute_waits(ev)
        self._job = _PushJob(list(self.client.links), ev, self.client.global_step, self.timing,
                             self._comm)
        self._pull_events = None
        self._fenced = 0
        from .. import ops
        ops.set_param_fence(self._op_fence)
        # the answer to this push is still in flight: report the step it will at least produce
        # (an async push advances the PS's global step by exactly one), or the owner's current
        # published step when other workers' pushes moved it further (one shared-memory read)
        return max(self.client.global_step + 1, self.client.links[0].global_step)

    # -- pull (next forward)
    def _issue_pulls(self):
        job, self._job = self._job, None
        t0 = time.perf_counter()
        self.client.global_step = job.result()          # raises the comm thread's error
        self.timing["fence_ms"].append((time.perf_counter() - t0) * 1e3)
        n = len(self.buckets)
        order = ([n - 1] + list(range(n - 2, -1, -1))) if self.space.decay_end < \
            self.space.numel else list(range(n - 1, -1, -1))
        events = [None] * n
        st = self._streams
        with st.side(), torch.no_grad():
            for b in order:
                s, e, _ = self.buckets[b]
                for link in self.client.links:
                    link.pull(self.space, s, e)
                events[b] = st.record()
        self._pull_events = events

    @comm_call
    def _wait_bucket(self, b):
        if self._job is not None:
            self._issue_pulls()
        evs = self._pull_events
        if evs is None or evs[b] is None:
            return
        self._streams.compute_waits(evs[b])
        evs[b] = None
        self._fenced += 1
        if self._fenced == len(evs):
            from .. import ops
            ops.set_param_fence(None)
            self._pull_events = None

    def _op_fence(self, args, kw):
        for a in list(args) + list(kw.values()):
            b = getattr(a, "_dtf_gbucket", None)
            if b is not None:
                self._wait_bucket(b)

    def _module_fence(self, module, _inputs):
        if self._job is not None or self._pull_events is not None:
            for p in module._parameters.values():
                b = getattr(p, "_dtf_gbucket", None)
                if b is not None:
                    self._wait_bucket(b)

    def drain(self):
        """Complete the push in flight and its pull (checkpoint, evaluation, end of training)."""
        if self._job is not None or self._pull_events is not None:
            for b in range(len(self.buckets)):
                self._wait_bucket(b)

    def reset_pipeline(self, join_s=5.0):
        """The cluster is being re-formed (recovery): whatever is in flight targets the old PS.
        Cancel and join the push in flight (bounded), drain the side stream so no copy into the
        old shard's mappings is still running, retire this generation's comm thread and detach
        the fences and the module pre-hook.  The next ``apply_remote`` starts generation + 1."""
        job, self._job = self._job, None
        if job is not None and not job.cancel(join_s):
            print(f"[dtf] pipelined push of global step {job.step} still blocked {join_s:g} s "
                  f"after cancel; its comm thread is abandoned", flush=True)
        if self._comm is not None:
            self._comm.retire()
            self._comm = None
        if self._streams is not None:
            self._streams.synchronize()
            self._streams = None
        self._pull_events, self._fenced, self._pipe = None, 0, None
        self._pushed_version = None
        # the interrupted step's buckets went to the old shard: the retried step (whose
        # begin_step skips the reset while the mode is undecided) must push every bucket again
        self.pending = [len(m) for (_, _, m) in self.buckets]
        self.launched = [False] * len(self.buckets)
        if self._pre_hook is not None:
            self._pre_hook.remove()
            self._pre_hook = None
        self.generation += 1
        from .. import ops
        ops.set_param_fence(None)

    def close(self, abort=False):
        if not abort:
            self.drain()
        self.reset_pipeline()
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for v in self.space.order:
            v._dtf_gbucket = None


def pipeline_enabled(device):
    """``DTF_PS_PIPELINE``: unset = on (GPU and CPU tasks), ``0`` = the serial data plane."""
    return os.environ.get("DTF_PS_PIPELINE", "1") != "0"


class _DoneEvent:
    """CPU stand-in for a HIP event: CPU copies have completed when they return."""

    @staticmethod
    def synchronize():
        pass

    @staticmethod
    def query():
        return True


class _Streams:
    """Stream/event operations of the pipelined data plane: a HIP side stream and events on a
    GPU; on a CPU task every copy is synchronous and in program order, so the side stream is
    the caller's thread and every event is complete when recorded."""

    def __init__(self, device):
        self.device = device
        self.cuda = device.type == "cuda"
        self.stream = torch.cuda.Stream(device) if self.cuda else None

    def side(self):
        import contextlib
        return torch.cuda.stream(self.stream) if self.cuda else contextlib.nullcontext()

    def side_waits_compute(self):
        if self.cuda:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))

    def record(self):
        if not self.cuda:
            return _DoneEvent()
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return ev

    def compute_waits(self, ev):
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_event(ev)

    def synchronize(self):
        if self.cuda:
            self.stream.synchronize()


class _PushJob:
    """One pipelined push on a generation's comm thread: wait for the mailbox copies, post to
    every owner, wait for their answers (the new global step).  ``cancel`` makes the answer
    wait give up at its next 200 ms slice; ``result`` is bounded by the links' own deadline."""

    def __init__(self, links, event, step, timing, thread):
        self.links, self.event, self.step, self.timing = links, event, step, timing
        self._done = threading.Event()
        self._cancelled = threading.Event()
        self._error = None
        self._step_out = None
        self._t0 = time.perf_counter()
        # the answer waits give up at the links' deadline; the host wait here a little later
        self.deadline_s = max((lk.timeout_ms for lk in links), default=0) / 1000.0 + 10.0
        thread.submit(self._run)

    def _run(self):
        try:
            if self._cancelled.is_set():
                raise ConnectionError(f"push of global step {self.step} cancelled before "
                                      f"posting (the cluster is re-forming)")
            self.event.synchronize()
            for link in self.links:
                link.post(self.step)
            steps = [link.wait(cancelled=self._cancelled.is_set) for link in self.links]
            self._step_out = steps[0]
            self.timing["answer_ms"].append((time.perf_counter() - self._t0) * 1e3)
        except BaseException as e:      # re-raised on the main thread at the fence
            self._error = e
        finally:
            self._done.set()

    def result(self):
        if not self._done.wait(self.deadline_s):
            raise TimeoutError(f"pipelined push of global step {self.step}: no answer from the "
                               f"parameter server(s) within {self.deadline_s:.0f} s")
        if self._error is not None:
            raise self._error
        return self._step_out

    def cancel(self, join_s):
        """Cancel and wait up to ``join_s`` for the comm thread to let go; True when it did."""
        self._cancelled.set()
        return self._done.wait(join_s)


class _CommThread:
    """One DAEMON thread running one generation's pipelined pushes in order (a
    ThreadPoolExecutor's workers are joined at interpreter exit: a push whose answer never comes
    would hang the exit).  ``retire`` ends it after the job it is running."""

    def __init__(self, name="dtf-ps-push"):
        import queue
        self.q = queue.Queue()
        self.t = threading.Thread(target=self._run, name=name, daemon=True)
        self.t.start()

    def _run(self):
        while True:
            fn = self.q.get()
            if fn is None:
                return
            fn()

    def submit(self, fn):
        self.q.put(fn)

    def retire(self):
        self.q.put(None)


def _bucket_plan(space, bucket_bytes):
    """Contiguous variable-aligned ranges of the flat buffer, ~``bucket_bytes`` each:
    [(start, end, [variable indices])]."""
    out, offs, n = [], space.offsets, len(space.order)
    cur, members = None, []
    for i in range(n):
        if cur is None:
            cur = offs[i]
        members.append(i)
        end = offs[i + 1] if i + 1 < n else space.numel
        if (end - cur) * 4 >= bucket_bytes or i + 1 == n:
            out.append((cur, end, members))
            cur, members = None, []
    return out


class _ColocatedPSReducer(BucketedAllReduce):
    """Colocated sync PS on RCCL: push overlapped with backward, pull overlapped with forward.

    The gradient buffer is cut into the same buckets as MirroredStrategy's all-reduce.

    * **Sharded owners** (``num_ps == world``, an elementwise optimizer, every bucket a multiple
      of ``world`` elements -- always true for world 1/2/4/8, the flat layout pads every variable
      to 64 elements): rank ``r`` owns chunk ``r`` of EVERY bucket.  When a bucket's last
      gradient lands (post-accumulate hook, during backward) ONE in-place
      ``reduce_scatter_tensor`` sums it into the owners' chunks (the gradient push of the
      reference's ``SyncReplicasOptimizer``, ``templates/00_mnist_replica.py:168-191``); after
      backward each owner runs the fused optimizer on its chunks, then ONE in-place
      ``all_gather_into_tensor`` per bucket hands the updated fp32 masters to every rank (the
      variable pull).  Equal chunks balance the update work and the link traffic exactly.
    * **Owner ranges** (``num_ps < world`` -- "1 PS + N workers" --, or a non-elementwise
      optimizer such as LAMB): variable-aligned owner slices; each owner's piece of a bucket is
      ``reduce``d to it, and the owner ``broadcast``s its updated piece.

    The pulls are launched last-layer-bucket LAST (the forward needs the first layers first) and
    are NOT waited for after the step: each bucket's wait is deferred to the first op of the next
    forward that reads one of its variables (``ops`` variable fence + a module forward pre-hook),
    so the gather of late layers overlaps the early layers' compute.  ``begin_step`` (before the
    next backward) and :meth:`drain` complete whatever the forward did not touch."""

    applies_update = True

    def __init__(self, space, owners_ranges, group=None, bucket_bytes=64 << 20,
                 first_bucket_bytes=4 << 20, sharded=None, overlap_gather=True, comm=None):
        super().__init__(space, group, bucket_bytes, first_bucket_bytes, comm=comm)
        self.rank = dist.get_rank(group)
        W = self.world
        ok = all((e - s) % W == 0 for s, e, _ in self.buckets) and \
            getattr(space, "elementwise", True)
        self.sharded = ok if sharded is None else (sharded and ok)
        if self.sharded:
            self.ranges = []
            self.pieces = []
            for s, e, _ in self.buckets:
                c = (e - s) // W
                self.pieces.append([(o, s + o * c, s + (o + 1) * c) for o in range(W)])
                self.ranges.append((self.rank, s + self.rank * c, s + (self.rank + 1) * c))
        else:
            self.ranges = owners_ranges          # [(owner_rank, start, end)]
            # per bucket: [(owner, start, end)] pieces (bucket ∩ owner range)
            self.pieces = []
            for bs, be, _ in self.buckets:
                self.pieces.append([(o, max(bs, s), min(be, e)) for o, s, e in owners_ranges
                                    if min(be, e) > max(bs, s)])
        self.overlap_gather = overlap_gather
        self.gpending = [None] * len(self.buckets)
        self._n_pending = 0
        for b, (_, _, mem) in enumerate(self.buckets):
            for i in mem:
                space.order[i]._dtf_gbucket = b
        self._pre_hook = None
        if overlap_gather:
            from torch.nn.modules.module import register_module_forward_pre_hook
            self._pre_hook = register_module_forward_pre_hook(self._module_fence)

    # -- push (during backward)
    @comm_call
    def _launch(self, b):
        if self.launched[b]:
            return
        self.launched[b] = True
        self.launch_log.append(b)
        g = self.space.grad
        if self.sharded:
            s, e, _ = self.buckets[b]
            _, cs, ce = self.pieces[b][self.rank]
            self.works.append((self.comm.reduce_scatter(g[cs:ce], g[s:e]), None, None))
            return
        for o, s, e in self.pieces[b]:
            self.works.append((self.comm.reduce(g[s:e], o), None, None))

    def grad_scale(self):
        return 1.0 / self.world

    # -- owner apply + pull
    @comm_call
    def apply_remote(self, optimizer):
        self.drain()
        for o, s, e in self.ranges:
            if o == self.rank and e > s:
                optimizer._apply(self.grad_scale(), (s, e))
        m = self.space.master
        # forward order: the non-decayed tail (BN / bias variables of every layer) first, then
        # the decayed buckets from the first layers (last bucket) to the last layers (bucket 0)
        n = len(self.buckets)
        order = ([n - 1] + list(range(n - 2, -1, -1))) if self.space.decay_end < \
            self.space.numel else list(range(n - 1, -1, -1))
        for b in order:
            if self.sharded:
                s, e, _ = self.buckets[b]
                _, cs, ce = self.pieces[b][self.rank]
                works = [self.comm.all_gather(m[s:e], m[cs:ce])]
            else:
                works = [self.comm.broadcast(m[s:e], o) for o, s, e in self.pieces[b]]
            self.gpending[b] = works
            self._n_pending += 1
        if self.overlap_gather:
            from .. import ops
            ops.set_param_fence(self._op_fence)
        else:
            self.drain()
        return None

    @comm_call
    def _wait_gather(self, b):
        works = self.gpending[b]
        if works is None:
            return
        self.gpending[b] = None
        for w in works:
            w.wait()
        sh = self.space.shadow
        if sh is not None:
            # through .data: the forward may already have saved bf16 weight views of this
            # buffer for backward, and a tracked in-place copy would bump their shared version
            # counter (autograd would then refuse the backward)
            s, e, _ = self.buckets[b]
            sh.data[s:e].copy_(self.space.master.data[s:e])
        self._n_pending -= 1
        if self._n_pending == 0:
            from .. import ops
            ops.set_param_fence(None)

    def _op_fence(self, args, kw):
        for a in args:
            b = getattr(a, "_dtf_gbucket", None)
            if b is not None and self.gpending[b] is not None:
                self._wait_gather(b)
        for a in kw.values():
            b = getattr(a, "_dtf_gbucket", None)
            if b is not None and self.gpending[b] is not None:
                self._wait_gather(b)

    def _module_fence(self, module, _inputs):
        if self._n_pending:
            for p in module._parameters.values():
                b = getattr(p, "_dtf_gbucket", None)
                if b is not None and self.gpending[b] is not None:
                    self._wait_gather(b)

    def drain(self):
        if self._n_pending:
            for b in range(len(self.buckets)):
                self._wait_gather(b)

    def begin_step(self):
        self.drain()
        super().begin_step()

    @comm_call
    def gather_state(self, bufs):
        """Sharded owners keep each slot chunk only on its owner: all-gather every slot buffer
        (collective; before a checkpoint of the slots)."""
        self.drain()
        for buf in bufs:
            for b, (s, e, _) in enumerate(self.buckets):
                if self.sharded:
                    _, cs, ce = self.pieces[b][self.rank]
                    self.comm.all_gather(buf[s:e], buf[cs:ce]).wait()
                else:
                    for o, ps, pe in self.pieces[b]:
                        self.comm.broadcast(buf[ps:pe], o).wait()

    def close(self, abort=False):
        """Detach hooks and fences.  ``abort``: the process group broke (a peer died) -- drop
        the pending variable gathers instead of waiting for them."""
        if abort:
            self.gpending = [None] * len(self.buckets)
            self._n_pending = 0
            from .. import ops
            ops.set_param_fence(None)
        else:
            self.drain()
        super().close()
        if self._pre_hook is not None:
            self._pre_hook.remove()
            self._pre_hook = None
        for v in self.space.order:
            v._dtf_gbucket = None


def balanced_ranges(space, num_owners, owner_ranks):
    """Contiguous, variable-aligned slices of the flat buffer with ~equal element counts."""
    total = space.numel
    bounds, target, k = [0], total / num_owners, 1
    for o in space.offsets[1:]:
        if k < num_owners and o >= target * k:
            bounds.append(o)
            k += 1
    while len(bounds) < num_owners:
        bounds.append(total)
    bounds.append(total)
    return [(owner_ranks[i], bounds[i], bounds[i + 1]) for i in range(num_owners)]


class ParameterServerStrategy(Strategy):
    def __init__(self, cluster_resolver=None, server=None, num_ps=None, sync=None,
                 replicas_to_aggregate=None, variable_placement="balanced", device=None,
                 data_plane=None, bucket_mb=64, first_bucket_mb=4, force_reducer=None,
                 sharded=None, overlap_gather=True, comm=None):
        self.server = server
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.first_bucket_bytes = int(first_bucket_mb * (1 << 20))
        self.data_plane = data_plane
        self.variable_placement = variable_placement
        self.replicas_to_aggregate = replicas_to_aggregate
        self.force_reducer = force_reducer_default() if force_reducer is None else force_reducer
        self.sharded = sharded
        self.overlap_gather = overlap_gather
        self.comm_kind = comm
        self._comm = None
        self._client = None
        if server is not None:
            # between-graph: this process is a worker of a PS cluster
            local = int(os.environ.get("LOCAL_RANK", "0"))
            if device is None:
                device = (torch.device("cuda", local % max(torch.cuda.device_count(), 1))
                          if torch.cuda.is_available() else torch.device("cpu"))
            if device.type == "cuda":
                torch.cuda.set_device(device)
            super().__init__(device)
            self.sync = bool(sync)
            self.mode = "between_graph"
        else:
            local = int(os.environ.get("LOCAL_RANK", "0"))
            if torch.cuda.is_available():
                torch.cuda.set_device(local)
                device = torch.device("cuda", local)
            else:
                device = torch.device("cpu")
            super().__init__(device)
            if int(os.environ.get("WORLD_SIZE", "1")) > 1 or self.force_reducer:
                init_process_group_from_env()
            self.sync = True if sync is None else bool(sync)
            if not self.sync:
                raise ValueError("colocated ParameterServerStrategy is synchronous; use a "
                                 "between-graph cluster (Server with ps tasks) for async PS")
            self.mode = "colocated"
            w = dist.get_world_size() if dist.is_initialized() else 1
            self.num_ps = min(num_ps or w, w)

    # -- topology
    @property
    def num_replicas_in_sync(self):
        if self.mode == "between_graph":
            return len(self.server.worker_ranks()) if self.sync else 1
        return dist.get_world_size() if dist.is_initialized() else 1

    @property
    def replica_id(self):
        if self.mode == "between_graph":
            return self.server.worker_ranks().index(self.server.rank)
        return dist.get_rank() if dist.is_initialized() else 0

    @property
    def is_chief(self):
        return self.server.is_chief if self.mode == "between_graph" else self.replica_id == 0

    # -- hooks used by Optimizer.build
    def make_gradient_reducer(self, space):
        if self.mode == "between_graph":
            from .ps_service import PSClient
            self._client = PSClient(self.server.ps_ranks(), policy=self.variable_placement,
                                    space=space, data_plane=self.data_plane,
                                    single_host=self.server.cluster.single_host())
            return _RemotePSReducer(space, self._client, sync=self.sync)
        if not self.collective:
            return _NullReducer(space)
        ranges = balanced_ranges(space, self.num_ps, list(range(self.num_ps)))
        sharded = (self.num_ps == dist.get_world_size()) and self.sharded is not False
        if self._comm is None:
            from .comm import make_comm
            self._comm = make_comm(self.comm_kind, None, self.device)
        return _ColocatedPSReducer(space, ranges, None, self.bucket_bytes,
                                   self.first_bucket_bytes, sharded=sharded,
                                   overlap_gather=self.overlap_gather, comm=self._comm)

    @property
    def collective(self):
        return self.mode == "colocated" and dist.is_initialized() and \
            (dist.get_world_size() > 1 or self.force_reducer)

    def sync_after_restore(self, optimizer, global_step=None, restored=False):
        _broadcast_training_state(self.collective, optimizer, global_step, restored=restored)

    def cluster_changed(self):
        if self.mode == "between_graph":
            return self.server.cluster_changed()
        return collective_cluster_changed()

    def broadcast_space(self, space):
        if self.collective:
            dist.broadcast(space.master, 0)
            space.refresh_shadow()

    def register_with_ps(self, optimizer, global_step=0, restored_slots=False, timeout_s=None):
        """Chief: ship variables + optimizer config (+ the optimizer slots just restored from a
        checkpoint) to the PS shards; others: wait for it."""
        if self.mode != "between_graph":
            return
        params = optimizer.space.order
        if self.is_chief:
            slots = None
            if restored_slots and optimizer.slots:
                slots = {s.name: [optimizer.space.view_of(s.buf, p) for p in params]
                         for s in optimizer.slots}
            self._client.register(params, optimizer.get_config(), sync=self.sync,
                                  replicas_to_aggregate=self.replicas_to_aggregate,
                                  global_step=int(global_step), slots=slots,
                                  iterations=optimizer.iterations if restored_slots else None)
        self._client.wait_ready(params, timeout_s)
        self._client.pull()          # every worker starts from the PS values

    def recover_cluster(self, optimizer):
        """A task of the cluster died (a PS crashed and is being restarted by the launcher):
        leave the broken process group, join the next generation (blocks until the restarted
        PS joins too) and re-map the new shard's buffers.  The caller restores the checkpoint
        and calls :meth:`register_with_ps` again (chief re-initialises the PS; others wait)."""
        if self.mode != "between_graph":
            # colocated owners: the same world re-formation as MirroredStrategy
            if self._comm is not None:
                try:
                    self._comm.close(abort=True)
                except Exception:
                    pass
                self._comm = None
            epoch = rejoin_collective()
            if optimizer is not None and optimizer.space is not None:
                old = optimizer._reducer
                if hasattr(old, "close"):
                    old.close(abort=True)
                optimizer._reducer = self.make_gradient_reducer(optimizer.space)
                self.broadcast_space(optimizer.space)     # mirrors the restarted rank's build
            return epoch
        reducer = getattr(optimizer, "_reducer", None)
        if reducer is not None and hasattr(reducer, "reset_pipeline"):
            # before leaving the group: cancel + join the push in flight (it targets the dead
            # generation's control block), drain the side stream, retire the comm thread
            reducer.reset_pipeline()
        self.server.restart_group()
        from .ps_service import PSClient
        old = self._client
        self._client = PSClient(self.server.ps_ranks(), policy=self.variable_placement,
                                space=old.space, data_plane=self.data_plane,
                                single_host=self.server.cluster.single_host())
        if reducer is not None and hasattr(reducer, "client"):
            reducer.client = self._client
        return self.server.generation

    @property
    def ps_client(self):
        return self._client

    def barrier(self):
        if self.mode == "colocated" and dist.is_initialized():
            dist.barrier()


# tf.compat.v1 naming
ParameterServerStrategyV1 = ParameterServerStrategy
CentralStorageStrategy = MirroredStrategy
