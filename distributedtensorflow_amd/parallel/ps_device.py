"""Device-resident parameter-server data plane (between-graph PS, the reference's primary mode).

Reference behaviour: every ``mon_sess.run`` of a worker pulls
the PS variables and pushes its gradients to the PS, which runs ``ApplyAdam`` on arrival (async,
Hogwild) or after ``replicas_to_aggregate`` fresh gradients (``SyncReplicasOptimizer``)
(``/root/reference/run_mnist_distributed.py:107-116,142-161``,
``/root/reference/templates/00_mnist_replica.py:168-191``).  TF1 moves every one of those tensors
through gRPC; round 1 of this framework moved them through host gloo/TCP.

MI355X design: the bytes never leave HBM and never pass through either process.

* The PS task (``Server.join()``) owns its variable shard as ONE flat fp32 buffer in its GPU's
  HBM plus one gradient mailbox slot per worker, all ``hipMalloc``-ed and exported with
  ``hipIpcGetMemHandle`` (``csrc/kernels/ipc.cpp``).
* A worker maps them with ``hipIpcOpenMemHandle``: on an 8-GPU node this is a peer mapping over
  xGMI (the worker's copy engines write its gradient straight into the owner's mailbox and read
  the fresh variables straight out of the owner's HBM), on a one-GPU box a second mapping of the
  same HBM.  A push is one device copy per contiguous shard; so is a pull.
* Signalling is a shared-memory control block of sequence words with futex sleep/wake
  (``csrc/native/shm_ctl.cpp``): post -> the owner's service thread wakes, runs the fused
  TF-exact optimizer kernel on the mailbox slot ON ITS OWN HIP STREAM, publishes the new
  global step and answers.  Sync mode holds the answers of a step's contributors until
  ``replicas_to_aggregate`` fresh gradients have been summed (stale ones are dropped at once):
  TF's ConditionalAccumulator + token queue.
* CPU tasks (tests, BASELINE config 1) run the identical protocol with the buffers in
  ``/dev/shm`` files instead of HBM.

The gloo world of ``Server`` stays the CONTROL plane (registration, checkpoint state, stop).
"""
from __future__ import annotations

import json
import os
import socket
import threading
import time
import uuid

import torch

ALIGN = 64   # elements; FlatSpace's per-variable alignment


# ----------------------------------------------------------------------------- shared buffers

def _native():
    from .._lib import _dtf_native
    return _dtf_native


def _hip():
    from ..ops import native
    return native.kernels()


# buffers this process exported: a mapping request from the SAME process (an owner and a worker
# colocated in one process, e.g. the data-plane tests) gets the original tensor -- HIP refuses to
# open an IPC handle in the process that created it
_LOCAL_EXPORTS = {}


def alloc_shared(numel, device, tag):
    """A zeroed fp32 buffer other processes of this node can map.  Returns (tensor, descriptor)."""
    device = torch.device(device)
    numel = max(int(numel), 1)
    if device.type == "cuda":
        from torch.utils.dlpack import from_dlpack
        cap, handle = _hip().ipc_alloc(numel, device.index or 0)
        t = from_dlpack(cap)
        _LOCAL_EXPORTS[handle.hex()] = t
        return t, {"kind": "ipc", "handle": handle.hex(), "numel": numel}
    path = f"/dev/shm/dtf_{tag}_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    with open(path, "wb") as f:
        f.truncate(numel * 4)
    t = torch.from_file(path, shared=True, size=numel, dtype=torch.float32)
    return t, {"kind": "shm", "path": path, "numel": numel}


def open_shared(desc, device):
    device = torch.device(device)
    if desc["kind"] == "ipc":
        if device.type != "cuda":
            raise RuntimeError("a CPU worker cannot map a parameter server's HBM shard")
        local = _LOCAL_EXPORTS.get(desc["handle"])
        if local is not None:
            return local
        from torch.utils.dlpack import from_dlpack
        return from_dlpack(_hip().ipc_open(bytes.fromhex(desc["handle"]), int(desc["numel"]),
                                           device.index or 0))
    return torch.from_file(desc["path"], shared=True, size=int(desc["numel"]),
                           dtype=torch.float32)


def release_shared(desc):
    if desc and desc.get("kind") == "ipc":
        _LOCAL_EXPORTS.pop(desc["handle"], None)
    if desc and desc.get("kind") == "shm":
        try:
            os.unlink(desc["path"])
        except FileNotFoundError:
            pass


# ----------------------------------------------------------------------------- layouts

def shard_plan(space, num_ps, policy="balanced"):
    """Which variables each PS owns, and where they live in the owner's flat buffer.

    ``balanced`` (default): contiguous, variable-aligned, ~equal-size slices of the worker's
    flat buffer, so a push / pull is ONE device copy per PS.  ``round_robin``: TF
    ``replica_device_setter`` parity (variable i -> ps i % num_ps; SURVEY §2.5 notes it puts
    99.97 % of the CNN's bytes on ps0), one copy per variable run.

    Returns per PS: {"vars": [i...], "owner_offsets": [...], "numel": n,
    "segments": [(worker_off, owner_off, length)]} (segments merged where contiguous)."""
    order, offs = space.order, space.offsets
    n = len(order)
    if policy == "round_robin":
        owner = [i % num_ps for i in range(n)]
    elif policy == "balanced":
        total = space.numel
        bounds, k = [0], 1
        for i, o in enumerate(offs):
            if k < num_ps and o >= total * k / num_ps and i > 0:
                bounds.append(i)
                k += 1
        while len(bounds) < num_ps:
            bounds.append(n)
        bounds.append(n)
        owner = [0] * n
        for k in range(num_ps):
            for i in range(bounds[k], bounds[k + 1]):
                owner[i] = k
    else:
        raise ValueError(policy)
    plans = []
    for k in range(num_ps):
        idx = [i for i in range(n) if owner[i] == k]
        oo, cur, segs = [], 0, []
        for i in idx:
            m = order[i].numel()
            oo.append(cur)
            if segs and offs[i] - segs[-1][0] == cur - segs[-1][1]:
                segs[-1][2] = offs[i] - segs[-1][0] + m      # same gaps on both sides: extend
            else:
                segs.append([offs[i], cur, m])
            cur += -(-m // ALIGN) * ALIGN
        plans.append({"vars": idx, "owner_offsets": oo, "numel": max(cur, 1),
                      "segments": [tuple(s) for s in segs]})
    return plans


class LayoutSpace:
    """FlatSpace-compatible view of a PS shard: variables live at given offsets of ONE flat
    master buffer (the exported HBM shard).  ``grad`` is re-pointed at the mailbox slot (async)
    or the aggregation buffer (sync) for each apply, so the optimizer kernels read the pushed
    gradient where it landed."""

    def __init__(self, master, names, shapes, offsets, decay):
        self.master = master
        self.numel = master.numel()
        self.device = master.device
        self.grad = None
        self.shadow = None
        self.order, self.offsets = [], list(offsets)
        for name, shape, o, dec in zip(names, shapes, offsets, decay):
            n = 1
            for d in shape:
                n *= d
            p = torch.nn.Parameter(master[o:o + n].view(shape), requires_grad=True)
            p._dtf_name = name
            p._dtf_decay = bool(dec)
            self.order.append(p)
        plain = [o for o, d in zip(offsets, decay) if not d]
        self.decay_end = min(plain) if plain else self.numel
        self.index = {id(v): i for i, v in enumerate(self.order)}

    def zero_grad(self):
        pass

    def refresh_shadow(self):
        pass

    def new_slot(self, fill=0.0):
        return torch.full((self.numel,), float(fill), device=self.device, dtype=torch.float32)

    def view_of(self, buf, v):
        i = self.index[id(v)]
        o = self.offsets[i]
        return buf[o:o + v.numel()].view(v.shape)

    def regions(self):
        out = [(0, self.decay_end, True)]
        if self.decay_end < self.numel:
            out.append((self.decay_end, self.numel, False))
        return [r for r in out if r[1] > r[0]]


def _make_optimizer(cfg, space):
    from ..optimizers import (AdagradOptimizer, AdamOptimizer, GradientDescentOptimizer,
                              LAMBOptimizer, MomentumOptimizer)
    from .strategy import _NullReducer
    cfg = dict(cfg)
    kind = cfg.pop("type")
    cls = {"adam": AdamOptimizer, "adagrad": AdagradOptimizer, "momentum": MomentumOptimizer,
           "sgd": GradientDescentOptimizer, "lamb": LAMBOptimizer}[kind]
    opt = cls(**cfg)
    opt.decay_filter = lambda v: getattr(v, "_dtf_decay", True)
    opt.space = space
    opt._build_slots()
    opt._lr_dev = torch.zeros(4, device=space.device, dtype=torch.float32)
    opt._nonfinite = torch.zeros(1, device=space.device, dtype=torch.int32)
    opt._reducer = _NullReducer(space)
    return opt


# ----------------------------------------------------------------------------- PS side

class OwnerShard:
    """A PS task's shard on the device data plane + its service thread.

    Streams (GPU shard).  Every write into the shard's buffers -- the initial values, restored
    slots, the sync accumulator, every optimizer apply -- is issued on the shard's own HIP
    streams and the shard is synchronised before it is published to workers, so nothing the
    default stream does can race with the service's writes.

    Async (Hogwild, TF ``use_locking=False``, the reference's mode): each worker's mailbox slot
    has its OWN stream and its own copy of the per-apply hyper-parameter buffers, so the
    service thread launches a worker's apply the moment its post arrives, without a host lock
    around the kernel and without waiting for other workers' applies; a completion thread
    answers each worker when ITS apply's event has completed (so the worker's next pull sees its
    update).  ``use_locking=True`` (spec) serialises the applies on one stream instead.
    Sync (SyncReplicasOptimizer): gradients are summed on the shard stream; the answer to the
    step's contributors follows the apply's event."""

    def __init__(self, spec, values, device, worker_ranks, ps_index):
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.names = spec["names"]
        self.shapes = [tuple(s) for s in spec["shapes"]]
        offsets = spec["owner_offsets"]
        numel = int(spec["numel"])
        self.numel = numel
        self.worker_ranks = list(worker_ranks)
        nw = len(self.worker_ranks)
        tag = f"ps{ps_index}"
        cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if cuda else None
        self.use_locking = bool(spec.get("use_locking", False))
        self.streams = ([self.stream] * nw if self.use_locking else
                        [torch.cuda.Stream(self.device) for _ in range(nw)]) if cuda else []
        self.master, self.master_desc = alloc_shared(numel, self.device, tag + "m")
        self.mail, self.mail_desc = alloc_shared(numel * nw, self.device, tag + "g")
        with self._on(self.stream), torch.no_grad():
            for (o, shape), v in zip(zip(offsets, self.shapes), _split(values, self.shapes)):
                n = v.numel()
                self.master[o:o + n].copy_(v.reshape(-1).to(self.device, non_blocking=False))
            self.space = LayoutSpace(self.master, self.names, self.shapes, offsets,
                                     spec["decay"])
            self.params = self.space.order
            self.opt = _make_optimizer(spec["optimizer"], self.space)
            # per-slot copies of the buffers one apply reads/writes besides the shard itself
            self._hyper = [self._hyper_buffers() for _ in range(max(nw, 1))]
        self._sync_device()
        self.opt.iterations = int(spec.get("iterations", spec.get("global_step", 0)))
        self.sync = bool(spec.get("sync", False))
        self.replicas_to_aggregate = int(spec.get("replicas_to_aggregate") or nw)
        self.global_step = int(spec.get("global_step", 0))
        self.ctl_name = f"dtf_ps{ps_index}_{os.getpid()}_{uuid.uuid4().hex[:8]}"
        self.ctl = _native().ShmControl(self.ctl_name, True, nw)
        self.ctl.global_step = self.global_step
        self.lock = threading.Lock()           # host bookkeeping only (never held over a sync)
        self._acc = None
        self._acc_count = 0
        self._waiters = []
        self._stopped_workers = set()
        self.stats = {"applied": 0, "dropped_stale": 0, "pushes": 0, "aggregated": 0,
                      "apply_s": 0.0, "max_inflight": 0}
        self._inflight = 0
        self._thread = None
        self._done_thread = None
        self._done_q = None
        self._error = None

    # -- helpers
    def _on(self, stream):
        import contextlib
        return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    def _sync_device(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def _hyper_buffers(self):
        o = self.opt
        out = {"_lr_dev": o._lr_dev.clone(), "_nonfinite": o._nonfinite}
        for name in ("_hyper", "_norms"):          # LAMB
            if hasattr(o, name):
                out[name] = getattr(o, name).clone()
        return out

    # -- descriptors for the workers (WAIT_READY reply)
    def descriptor(self):
        self._sync_device()                   # every initial write landed before publishing
        return {"plane": "ipc" if self.master_desc["kind"] == "ipc" else "shm",
                "master": self.master_desc, "mail": self.mail_desc, "numel": self.numel,
                "ctl": self.ctl_name, "workers": self.worker_ranks,
                "global_step": self.global_step, "pid": os.getpid(),
                "host": socket.gethostname(),
                "device": self.device.index if self.device.type == "cuda" else None}

    # -- control-plane API shared with ps_service._Shard
    def flat_values(self):
        with self.lock:
            self._sync_device()
            return torch.cat([p.detach().reshape(-1) for p in self.params]).cpu()

    def _join_workers(self):
        """Order the shard stream after every worker stream's applies (async mode)."""
        if self.stream is not None:
            for s in self.streams:
                if s is not self.stream:
                    self.stream.wait_stream(s)

    def set_values(self, vals, global_step):
        self._join_workers()
        with self.lock, self._on(self.stream), torch.no_grad():
            for p, v in zip(self.params, _split(vals, self.shapes)):
                p.copy_(v.to(p.device))
            self.global_step = int(global_step)
            self.ctl.global_step = self.global_step
        self._sync_device()

    def load_slot(self, name, flat):
        """Restore one optimizer slot (e.g. ``Adam``) from an unpadded flat of the shard's
        variables (checkpoint restore after a PS restart)."""
        slot = next(s for s in self.opt.slots if s.name == name)
        self._join_workers()
        with self.lock, self._on(self.stream), torch.no_grad():
            for p, v in zip(self.params, _split(flat, self.shapes)):
                self.space.view_of(slot.buf, p).copy_(v.to(slot.buf.device))
        self._sync_device()

    def worker_stopped(self, worker_rank):
        with self.lock:
            self._stopped_workers.add(worker_rank)
            if self.sync and self._waiters and \
                    len(self._stopped_workers) + len(self._waiters) >= len(self.worker_ranks):
                self._close_step()

    # -- service thread
    def start(self):
        import queue
        self._sync_device()
        self._done_q = queue.Queue()
        self._done_thread = threading.Thread(target=self._answer, name="dtf-ps-answers",
                                             daemon=True)
        self._done_thread.start()
        self._thread = threading.Thread(target=self._serve, name="dtf-ps-dataplane",
                                        daemon=True)
        self._thread.start()

    def stop(self):
        self.ctl.stop()
        if self._thread is not None:
            self._thread.join(timeout=10)
        if self._done_q is not None:
            self._done_q.put(None)
            self._done_thread.join(timeout=10)
        self._sync_device()
        release_shared(self.master_desc)
        release_shared(self.mail_desc)
        self.ctl.unlink()

    def _serve(self):
        try:
            if self.stream is not None:
                torch.cuda.set_device(self.device)
            while True:
                got = self.ctl.wait_any(200)
                if got is None:
                    return
                self.ctl.beat()
                for w, step in got:
                    self._on_push(w, step)
        except Exception as e:   # surfaced through ParameterServerService
            import traceback
            traceback.print_exc()
            self._error = e
            self.ctl.stop()

    def _answer(self):
        """Completion thread: answer workers in launch order once their apply finished."""
        try:
            if self.stream is not None:
                torch.cuda.set_device(self.device)
            while True:
                item = self._done_q.get()
                if item is None:
                    return
                ev, t0, answers, step = item
                if ev is not None:
                    ev.synchronize()
                with self.lock:
                    self._inflight -= 1
                    self.stats["apply_s"] += time.perf_counter() - t0
                    if step is not None and step > int(self.ctl.global_step):
                        self.ctl.global_step = step
                for w, s in answers:
                    self.ctl.done(w, s)
        except Exception as e:
            import traceback
            traceback.print_exc()
            self._error = e
            self.ctl.stop()

    def _slot(self, w):
        return self.mail[w * self.numel:(w + 1) * self.numel]

    def _launch_apply(self, grad, scale, w, answers, step):
        """Fused TF-exact optimizer over the shard on worker ``w``'s stream, reading the gradient
        in place; ``answers`` are released by the completion thread after it finished."""
        t0 = time.perf_counter()
        stream = self.streams[w] if self.streams else None
        sp, opt = self.space, self.opt
        with self._on(stream):
            if stream is not None:
                # the mailbox was filled by the worker (host-synchronised before its post); the
                # accumulator by the shard stream
                stream.wait_stream(self.stream)
            for k, v in self._hyper[w].items():
                setattr(opt, k, v)
            sp.grad = grad
            try:
                opt.iterations += 1
                opt._apply(scale)
            finally:
                sp.grad = None
            ev = None
            if stream is not None:
                ev = torch.cuda.Event()
                ev.record(stream)
                if self.sync or self.use_locking:
                    self.stream.wait_stream(stream)  # later accumulator / state writes
                # Hogwild (async, use_locking=False): the next worker's apply must NOT queue
                # behind this one through the shard stream -- applies of different workers run
                # concurrently on their own streams (TF's unlocked ApplyMomentum); shard-stream
                # work (restore, reads) joins every worker stream first (_join_workers)
        self.stats["applied"] += 1
        self._inflight += 1
        self.stats["max_inflight"] = max(self.stats["max_inflight"], self._inflight)
        self._done_q.put((ev, t0, answers, step))

    def _maybe_fault(self):
        """DTF_FAULT_KILL_PS_AT_STEP=n (tests): this PS task dies (SIGKILL, no cleanup, like a
        preempted host) once its global step reaches n -- only in the first incarnation."""
        n = int(os.environ.get("DTF_FAULT_KILL_PS_AT_STEP", "0") or 0)
        if n and self.global_step >= n and not int(os.environ.get("DTF_RESTART_COUNT", "0")):
            import signal
            os.kill(os.getpid(), signal.SIGKILL)

    def _on_push(self, w, step):
        with self.lock:
            self.stats["pushes"] += 1
            if not self.sync:
                self.global_step += 1
                self._maybe_fault()
                self._launch_apply(self._slot(w), 1.0, w, [(w, self.global_step)],
                                   self.global_step)
                return
            if step < self.global_step:                  # stale gradient: drop, release now
                self.stats["dropped_stale"] += 1
                self.ctl.done(w, self.global_step)
                return
            slot = self._slot(w)
            if self._acc is None:
                with self._on(self.stream):
                    self._acc = torch.zeros_like(slot)
                self._acc_count = 0
            if self._acc_count < self.replicas_to_aggregate:
                with self._on(self.stream):
                    self._acc.add_(slot)
                self._acc_count += 1
                self.stats["aggregated"] += 1
            else:
                self.stats["dropped_stale"] += 1
            self._waiters.append(w)
            if self._acc_count >= self.replicas_to_aggregate:
                self._close_step()

    def _close_step(self):
        waiters, self._waiters = self._waiters, []
        if self._acc is not None and self._acc_count > 0:
            self.global_step += 1
            # the apply runs on the shard stream (slot 0's stream is the shard stream under
            # use_locking; otherwise the sync apply gets its own ordering via the shard stream)
            self._launch_apply(self._acc, 1.0 / self._acc_count, 0,
                               [(w, self.global_step) for w in waiters], self.global_step)
            with self._on(self.stream):
                self._acc.zero_()                # ordered after the apply (shard stream)
        else:
            for w in waiters:
                self.ctl.done(w, self.global_step)
        self._acc_count = 0


def _split(flat, shapes):
    out, off = [], 0
    for s in shapes:
        n = 1
        for d in s:
            n *= d
        out.append(flat[off:off + n].view(s))
        off += n
    return out


# ----------------------------------------------------------------------------- worker side

class PSLink:
    """A worker's mapping of one PS shard: its mailbox slot, the owner's variables, the control
    block.  ``push`` copies the shard's gradient into the mailbox and posts; ``wait`` returns
    the owner's new global step; ``pull`` copies the owner's variables into the local flat
    master buffer (and its bf16 compute shadow)."""

    def __init__(self, desc, plan, worker_index, device, ps_index, timeout_s=None):
        host = desc.get("host")
        if host is not None and host != socket.gethostname():
            raise RuntimeError(f"parameter server {ps_index} runs on host {host!r}, this worker "
                               f"on {socket.gethostname()!r}: its device data plane cannot be "
                               f"mapped here (use data_plane='gloo' across hosts)")
        self.desc = desc
        self.plan = plan
        self.w = int(worker_index)
        self.device = torch.device(device)
        self.ps_index = ps_index
        check_peer_access(desc, self.device, ps_index)
        self.owner_master = open_shared(desc["master"], self.device)
        mail = open_shared(desc["mail"], self.device)
        n = int(desc["numel"])
        self.slot = mail[self.w * n:(self.w + 1) * n]
        self._mail = mail
        self.ctl = _native().ShmControl(desc["ctl"], False, len(desc["workers"]))
        self.timeout_ms = int(1000 * (timeout_s if timeout_s is not None else
                                      float(os.environ.get("DTF_PS_TIMEOUT_S", "600"))))

    def _segments(self, lo=None, hi=None):
        """This shard's (worker offset, owner offset, length) runs, clipped to the worker's flat
        range [lo, hi) (one gradient / variable bucket)."""
        for wo, oo, n in self.plan["segments"]:
            if lo is None:
                yield wo, oo, n
                continue
            a, b = max(wo, lo), min(wo + n, hi)
            if b > a:
                yield a, oo + (a - wo), b - a

    def copy_grads(self, space, lo=None, hi=None):
        for wo, oo, n in self._segments(lo, hi):
            self.slot[oo:oo + n].copy_(space.grad[wo:wo + n], non_blocking=True)

    def post(self, step):
        self.ctl.post(self.w, int(step))

    def _owner_alive(self):
        pid = self.desc.get("pid")
        if not pid:
            return True
        try:
            os.kill(int(pid), 0)          # same host: signal 0 probes the PS task
        except ProcessLookupError:
            return False
        except PermissionError:
            return True
        # a SIGKILLed task stays a zombie until its parent (the launcher) reaps it, and signal 0
        # still succeeds on a zombie: read its state
        try:
            with open(f"/proc/{int(pid)}/stat") as f:
                state = f.read().rpartition(")")[2].split()[0]
            return state not in ("Z", "X")
        except (OSError, IndexError):
            return True

    def wait(self, cancelled=None):
        """The owner's answer (new global step).  Sleeps on the futex in 200 ms slices and
        probes the owner process between them, so a dead PS surfaces as ConnectionError at once
        (MonitoredTrainingSession recovers from it) instead of after the full timeout.
        ``cancelled()`` True (the pipelined plane's recovery) ends the wait at the next slice."""
        waited = 0
        while True:
            r = self.ctl.wait_done(self.w, 200)
            if r is not None:
                return int(r)
            waited += 200
            if cancelled is not None and cancelled():
                raise ConnectionError(f"wait for parameter server {self.ps_index}'s answer "
                                      f"cancelled (the cluster is re-forming)")
            if not self._owner_alive():
                raise ConnectionError(f"parameter server {self.ps_index} (pid "
                                      f"{self.desc.get('pid')}) died")
            if waited >= self.timeout_ms:
                raise ConnectionError(f"parameter server {self.ps_index} did not answer within "
                                      f"{self.timeout_ms / 1000:.0f} s (heartbeat "
                                      f"{self.ctl.heartbeat})")

    def pull(self, space, lo=None, hi=None):
        for wo, oo, n in self._segments(lo, hi):
            space.master[wo:wo + n].copy_(self.owner_master[oo:oo + n], non_blocking=True)
            if space.shadow is not None:
                space.shadow[wo:wo + n].copy_(space.master[wo:wo + n], non_blocking=True)

    @property
    def global_step(self):
        return int(self.ctl.global_step)


def check_peer_access(desc, device, ps_index=0):
    """A worker on GPU a mapping the HBM shard of an owner on GPU b != a reads and writes it
    over xGMI through the peer mapping ``hipIpcOpenMemHandle`` creates -- only possible when the
    two devices are peers.  Check first (``hipDeviceCanAccessPeer``) and fail with the reason
    instead of inside the IPC open or, worse, at the first copy."""
    owner = desc.get("device")
    if desc.get("master", {}).get("kind") != "ipc" or owner is None or device.type != "cuda":
        return
    mine = device.index if device.index is not None else torch.cuda.current_device()
    if int(owner) == mine:
        return
    if not torch.cuda.can_device_access_peer(mine, int(owner)):
        raise RuntimeError(f"parameter server {ps_index} keeps its shard on GPU {owner}, which "
                           f"GPU {mine} cannot access as a peer (hipDeviceCanAccessPeer = 0): "
                           f"put the PS task on a peer GPU, or use data_plane='gloo'")


def sync_device(device):
    device = torch.device(device)
    if device.type == "cuda":
        torch.cuda.current_stream(device).synchronize()


def spec_for(space, plan, names=None):
    order, offs = space.order, space.offsets
    return {"names": [names[i] if names else getattr(order[i], "_dtf_name", str(i))
                      for i in plan["vars"]],
            "shapes": [list(order[i].shape) for i in plan["vars"]],
            "owner_offsets": plan["owner_offsets"], "numel": plan["numel"],
            "decay": [offs[i] < space.decay_end for i in plan["vars"]]}


def dumps(d):
    return json.dumps(d).encode()
