"""Between-graph parameter-server engine (the reference's mode of operation).

Reference behaviour being reproduced:
  * ``ps`` tasks host the variables (``replica_device_setter``, ``run_mnist_distributed.py:107``)
    and block in ``server.join()`` (``:100-103``);
  * the chief worker initialises the variables on the PS, other workers wait
    (``MonitoredTrainingSession`` / ``Supervisor``, ``templates/00_mnist_replica.py:193-235``);
  * ASYNC (default): each worker pulls the current variables, computes gradients on its own
    batch and pushes them; the PS applies them on arrival without locks (Hogwild) and increments
    ``global_step`` — 1000 global steps are shared by all workers;
  * SYNC (``SyncReplicasOptimizer``, ``templates/00_mnist_replica.py:168-191``): the PS
    aggregates ``replicas_to_aggregate`` gradients computed at the current step (stale ones are
    dropped), averages them, applies once, increments the step and releases the waiting
    workers (the token queue);
  * variables are sharded over PS tasks: round-robin by variable (TF parity) or greedy
    byte-balanced (default; SURVEY §2.5 notes round-robin puts 99.97 % of the CNN on ps0).

Transport.  CONTROL plane: torch.distributed point-to-point on the ``gloo`` world (registration,
checkpoint state, stop/shutdown; any-source receives).  DATA plane (``ps_device.py``, default on
one node): the shard lives in the PS task's HBM (or a /dev/shm file for CPU tasks), workers map it
with hipIpc, write gradients into per-worker mailbox slots and read variables back with device
copies; a futex-signalled shared-memory control block replaces the per-step messages.  The
round-1 host path (every tensor ``.cpu()``-ed through gloo) remains as ``data_plane="gloo"``
for clusters that span hosts.

Clean shutdown (the reference's TODO, ``README.md:7``): workers send STOP when done; ``join()``
returns when every worker stopped, on SIGINT/SIGTERM, or on the chief's SHUTDOWN.
"""
from __future__ import annotations

import json
import signal
import threading
import time

import torch
import torch.distributed as dist

from .strategy import comm_call

OP_INIT, OP_PULL, OP_PUSH, OP_STOP, OP_WAIT_READY, OP_GET_STATE, OP_SET_STATE, OP_SHUTDOWN, \
    OP_GET_STEP = range(1, 10)
HDR = 8


def _hdr(*vals):
    t = torch.zeros(HDR, dtype=torch.int64)
    for i, v in enumerate(vals):
        t[i] = int(v)
    return t


def _send_bytes(b: bytes, dst, group=None):
    t = torch.frombuffer(bytearray(b), dtype=torch.uint8) if b else torch.zeros(0, dtype=torch.uint8)
    dist.send(torch.tensor([t.numel()], dtype=torch.int64), dst, group=group)
    if t.numel():
        dist.send(t, dst, group=group)


def _recv_bytes(src, group=None) -> bytes:
    n = torch.zeros(1, dtype=torch.int64)
    dist.recv(n, src, group=group)
    t = torch.zeros(int(n.item()), dtype=torch.uint8)
    if t.numel():
        dist.recv(t, src, group=group)
    return bytes(t.numpy().tobytes())


# ----------------------------------------------------------------------------- placement

def assign_shards(sizes, num_ps, policy="balanced"):
    """Owner PS index per variable.  ``round_robin`` = replica_device_setter parity;
    ``balanced`` = greedy largest-first onto the least-loaded PS (by element count)."""
    if num_ps <= 1:
        return [0] * len(sizes)
    if policy == "round_robin":
        return [i % num_ps for i in range(len(sizes))]
    if policy != "balanced":
        raise ValueError(policy)
    load = [0] * num_ps
    owner = [0] * len(sizes)
    for i in sorted(range(len(sizes)), key=lambda i: -sizes[i]):
        k = min(range(num_ps), key=lambda j: (load[j], j))
        owner[i] = k
        load[k] += sizes[i]
    return owner


def choose_plane(requested, ps_device):
    """Data plane of a PS shard: ``ipc`` (HBM shard, hipIpc-mapped by GPU workers) when the PS
    task has a GPU, ``shm`` (/dev/shm shard) for a CPU PS on the workers' host, ``gloo`` (host
    tensors over TCP, cross-host clusters) when asked for."""
    requested = requested or "gloo"
    if requested == "gloo":
        return "gloo"
    dev = torch.device(ps_device)
    if requested in ("auto", "ipc") and dev.type == "cuda":
        return "ipc"
    return "shm"


# ----------------------------------------------------------------------------- PS side

class _Shard:
    def __init__(self, spec, values, device):
        from ..optimizers import (AdagradOptimizer, AdamOptimizer, GradientDescentOptimizer,
                                  LAMBOptimizer, MomentumOptimizer)
        self.names = spec["names"]
        self.shapes = [tuple(s) for s in spec["shapes"]]
        self.numel = int(values.numel())
        self.device = device
        opt = dict(spec["optimizer"])
        kind = opt.pop("type")
        cls = {"adam": AdamOptimizer, "adagrad": AdagradOptimizer, "momentum": MomentumOptimizer,
               "sgd": GradientDescentOptimizer, "lamb": LAMBOptimizer}[kind]
        self.params = [torch.nn.Parameter(t.clone().to(device)) for t in
                       _split(values, self.shapes)]
        for p, n in zip(self.params, self.names):
            p._dtf_name = n
        self.opt = cls(**opt)
        from ..parallel import strategy as _st
        with _st.OneDeviceStrategy(device).scope():
            self.opt.build(self.params)
        self.opt.iterations = int(spec.get("iterations", spec.get("global_step", 0)))
        self.lock = threading.Lock()

    def load_slot(self, name, flat):
        slot = next(s for s in self.opt.slots if s.name == name)
        with self.lock, torch.no_grad():
            for p, v in zip(self.params, _split(flat, self.shapes)):
                self.opt.space.view_of(slot.buf, p).copy_(v.to(slot.buf.device))

    def flat_values(self):
        return torch.cat([p.detach().reshape(-1) for p in self.params]).cpu() if self.params \
            else torch.zeros(0)

    def apply(self, flat_grad, scale=1.0):
        with self.lock:
            sp = self.opt.space
            off = 0
            for p in self.params:
                n = p.numel()
                sp.view_of(sp.grad, p).copy_(flat_grad[off:off + n].view(p.shape))
                off += n
            self.opt.iterations += 1
            self.opt._apply(scale)


def _split(flat, shapes):
    out, off = [], 0
    for s in shapes:
        n = 1
        for d in s:
            n *= d
        out.append(flat[off:off + n].view(s))
        off += n
    return out


class ParameterServerService:
    """The loop run by ``Server.join()`` on a ``ps`` task."""

    def __init__(self, ps_index, worker_ranks, device="cpu", group=None, cluster_changed=None):
        self.ps_index = ps_index
        self.cluster_changed = cluster_changed
        self.worker_ranks = list(worker_ranks)
        self.device = torch.device(device)
        self.group = group
        self.shard = None
        self.sync = False
        self.replicas_to_aggregate = len(self.worker_ranks)
        self.global_step = 0
        self.stopped = set()
        self.waiting_ready = []
        self._acc = None
        self._acc_count = 0
        self._sync_waiters = []
        self._shutdown = False
        self.stats = {"applied": 0, "dropped_stale": 0, "pulls": 0}
        self.plane = "gloo"

    def _install_signal_handlers(self):
        def handler(signum, frame):
            self._shutdown = True
        for s in (signal.SIGINT, signal.SIGTERM):
            try:
                signal.signal(s, handler)
            except ValueError:   # not in main thread
                pass

    def serve(self):
        """Blocking any-source receives run on a service thread (gloo's ``is_completed`` is
        not updated for receives, so the loop cannot poll); the calling (main) thread keeps
        SIGINT/SIGTERM responsive and returns as soon as the service ends or is shut down."""
        from ..cluster import rendezvous
        self._install_signal_handlers()
        self._error = None
        rejoin = False
        t = threading.Thread(target=self._loop, name="dtf-ps-service", daemon=True)
        t.start()
        try:
            while t.is_alive() and not self._shutdown:
                t.join(timeout=0.2)
                dev_err = getattr(self.shard, "_error", None)
                if dev_err is not None:
                    raise dev_err
                if self.cluster_changed is not None and self.cluster_changed():
                    rejoin = True        # a peer died and was restarted: new epoch
                    break
            if self._error is not None and not rejoin:
                if rendezvous.recovery_enabled():
                    rejoin = True        # our group broke under a dead peer: restart with it
                else:
                    raise self._error
        finally:
            if self.plane != "gloo" and self.shard is not None:
                self.stats.update({k: v for k, v in self.shard.stats.items()})
                self.shard.stop()
        self.stats["global_step"] = self._gstep()
        self.stats["data_plane"] = self.plane
        self.stats["interrupted"] = t.is_alive()
        self.stats["rejoin"] = rejoin
        return self.stats

    def _gstep(self):
        return self.shard.global_step if self.plane != "gloo" and self.shard is not None \
            else self.global_step

    def _ready_reply(self, dst):
        if self.plane == "gloo":
            dist.send(_hdr(1, self.global_step, 0), dst, group=self.group)
        else:
            dist.send(_hdr(1, self._gstep(), 1), dst, group=self.group)
            _send_bytes(json.dumps(self.shard.descriptor()).encode(), dst, self.group)

    def _loop(self):
        hdr = torch.zeros(HDR, dtype=torch.int64)
        try:
            while not self._shutdown and len(self.stopped) < len(self.worker_ranks):
                dist.recv(hdr, group=self.group)
                self._dispatch(hdr.clone(), int(hdr[1]))   # every header carries its sender
        except Exception as e:  # surfaced by serve()
            self._error = e

    # -- handlers
    def _dispatch(self, h, src):
        op = int(h[0])
        if op == OP_INIT:
            spec = json.loads(_recv_bytes(src, self.group).decode())
            vals = torch.zeros(int(h[2]), dtype=torch.float32)
            dist.recv(vals, src, group=self.group)
            self.sync = bool(spec.get("sync", False))
            self.replicas_to_aggregate = int(spec.get("replicas_to_aggregate") or
                                             len(self.worker_ranks))
            self.global_step = int(spec.get("global_step", 0))
            self.plane = choose_plane(spec.get("data_plane", "gloo"), self.device)
            slot_vals = {}
            for sname in spec.get("slot_values", []):   # restored optimizer slots
                t = torch.zeros(vals.numel(), dtype=torch.float32)
                dist.recv(t, src, group=self.group)
                slot_vals[sname] = t
            if self.plane == "gloo":
                self.shard = _Shard(spec, vals, self.device)
            else:
                from .ps_device import OwnerShard
                self.shard = OwnerShard(spec, vals, self.device, self.worker_ranks,
                                        self.ps_index)
            for sname, t in slot_vals.items():
                self.shard.load_slot(sname, t)
            if self.plane != "gloo":
                self.shard.start()
            for w in self.waiting_ready:
                self._ready_reply(w)
            self.waiting_ready = []
        elif op == OP_WAIT_READY:
            if self.shard is None:
                self.waiting_ready.append(src)
            else:
                self._ready_reply(src)
        elif op == OP_PULL:
            self.stats["pulls"] += 1
            dist.send(_hdr(self.global_step, self.shard.numel), src, group=self.group)
            dist.send(self.shard.flat_values(), src, group=self.group)
        elif op == OP_PUSH:
            grad = torch.zeros(self.shard.numel, dtype=torch.float32)
            dist.recv(grad, src, group=self.group)
            step_of_grad = int(h[2])
            inc = int(h[3])     # 1 if this PS owns global_step (ps0)
            want = int(h[4])    # 1: reply with the updated values (push+pull in one trip)
            if not self.sync:
                self.shard.apply(grad.to(self.device))
                self.stats["applied"] += 1
                if inc:
                    self.global_step += 1
                self._reply_step(src, want)
            else:
                self._sync_push(src, grad, step_of_grad, inc, want)
        elif op == OP_GET_STEP:
            dist.send(_hdr(self._gstep()), src, group=self.group)
        elif op == OP_STOP:
            self.stopped.add(src)
            if self.plane != "gloo" and self.shard is not None:
                self.shard.worker_stopped(src)
            # a stopped worker must not hold the sync barrier of the others
            if self.sync and self._sync_waiters and \
                    len(self.stopped) + len(self._sync_waiters) >= len(self.worker_ranks):
                self._close_sync_step(force=True)
        elif op == OP_GET_STATE:
            st = {"global_step": self._gstep(), "names": self.shard.names,
                  "shapes": [list(s) for s in self.shard.shapes],
                  "slots": [s.name for s in self.shard.opt.slots],
                  "iterations": self.shard.opt.iterations}
            _send_bytes(json.dumps(st).encode(), src, self.group)
            dist.send(self.shard.flat_values(), src, group=self.group)
            for s in self.shard.opt.slots:
                dist.send(torch.cat([self.shard.opt.space.view_of(s.buf, p).reshape(-1)
                                     for p in self.shard.params]).cpu(), src, group=self.group)
        elif op == OP_SET_STATE:
            vals = torch.zeros(sum(_prod(sh) for sh in self.shard.shapes), dtype=torch.float32)
            dist.recv(vals, src, group=self.group)
            if self.plane != "gloo":
                self.shard.set_values(vals, int(h[2]))
                return
            with torch.no_grad():
                for p, v in zip(self.shard.params, _split(vals, self.shard.shapes)):
                    p.copy_(v)
            self.shard.opt.space.refresh_shadow()
            self.global_step = int(h[2])
        elif op == OP_SHUTDOWN:
            self._shutdown = True
        else:
            raise RuntimeError(f"PS {self.ps_index}: unknown op {op} from rank {src}")

    def _reply_step(self, dst, want_values):
        dist.send(_hdr(self.global_step, self.shard.numel), dst, group=self.group)
        if want_values:
            dist.send(self.shard.flat_values(), dst, group=self.group)

    def _sync_push(self, src, grad, step_of_grad, inc, want=0):
        if step_of_grad < self.global_step:          # stale: drop, release immediately
            self.stats["dropped_stale"] += 1
            self._reply_step(src, want)
            return
        if self._acc is None:
            self._acc = torch.zeros_like(grad)
            self._acc_count = 0
        if self._acc_count < self.replicas_to_aggregate:
            self._acc += grad
            self._acc_count += 1
        else:
            self.stats["dropped_stale"] += 1         # backup worker, step already full
        self._sync_waiters.append((src, want))
        self._inc = inc
        if self._acc_count >= self.replicas_to_aggregate:
            self._close_sync_step()

    def _close_sync_step(self, force=False):
        if self._acc is not None and self._acc_count > 0:
            self.shard.apply((self._acc / self._acc_count).to(self.device))
            self.stats["applied"] += 1
            if getattr(self, "_inc", 0):
                self.global_step += 1
        self._acc = None
        self._acc_count = 0
        waiters, self._sync_waiters = self._sync_waiters, []
        for w, want in waiters:
            self._reply_step(w, want)


# ----------------------------------------------------------------------------- worker side

class PSClient:
    """Worker-side view of the sharded PS variables.

    ``register(params, optimizer_cfg)`` (chief) / ``wait_ready()`` (others), then per step:
    ``pull()`` copies the PS values into the local parameters, ``push()`` sends the local
    gradients and returns the new global step."""

    def __init__(self, ps_ranks, group=None, policy="balanced", space=None, data_plane=None,
                 single_host=True):
        import os
        self.ps_ranks = list(ps_ranks)
        self.group = group
        self.policy = policy
        self.space = space
        # device data plane needs the flat buffers (ps_device.py); "gloo" = round-1 host path
        plane = (data_plane or os.environ.get("DTF_PS_DATA_PLANE", "auto")) \
            if space is not None else "gloo"
        if not single_host and plane != "gloo":
            # hipIpc / /dev/shm mappings only exist between processes of one host: a cluster
            # spanning hosts (the reference's config.json lists tasks by IP) uses TCP
            if plane != "auto":
                raise ValueError(f"data_plane={plane!r} needs every task on one host; this "
                                 f"cluster spans several (use 'auto' or 'gloo')")
            plane = "gloo"
        self.data_plane = plane
        self.params = None
        self.owner = None
        self.global_step = 0
        self.links = None
        self.plans = None
        # host-side time per push on the device plane (bench breakdown): waiting for the local
        # gradients + mailbox copy, waiting for the owner's answer, issuing the pull
        self.timing = {"copy_sync_ms": [], "wait_ms": [], "pull_ms": []}

    def _layout(self, params):
        self.params = list(params)
        if self.space is not None:
            from .ps_device import shard_plan
            self.plans = shard_plan(self.space, len(self.ps_ranks), self.policy)
            self.by_ps = [pl["vars"] for pl in self.plans]
            self.owner = [0] * len(self.params)
            for k, idx in enumerate(self.by_ps):
                for i in idx:
                    self.owner[i] = k
            return
        self.owner = assign_shards([p.numel() for p in self.params], len(self.ps_ranks),
                                   self.policy)
        self.by_ps = [[i for i, o in enumerate(self.owner) if o == k]
                      for k in range(len(self.ps_ranks))]

    @property
    def data_plane_in_use(self):
        return "gloo" if not self.links else self.links[0].desc.get("plane", "?")

    @comm_call
    def register(self, params, optimizer_cfg, names=None, sync=False, replicas_to_aggregate=None,
                 global_step=0, slots=None, iterations=None):
        """Chief: ship each shard's variables (and, on a restore, its optimizer slots:
        ``slots = {name: per-variable tensors aligned with params}``) to its PS."""
        self._layout(params)
        for k, rank in enumerate(self.ps_ranks):
            idx = self.by_ps[k]
            spec = {"names": [names[i] if names else getattr(self.params[i], "_dtf_name", str(i))
                              for i in idx],
                    "shapes": [list(self.params[i].shape) for i in idx],
                    "optimizer": optimizer_cfg, "sync": sync,
                    "replicas_to_aggregate": replicas_to_aggregate,
                    "global_step": global_step, "data_plane": self.data_plane,
                    "iterations": int(global_step if iterations is None else iterations),
                    "slot_values": sorted(slots) if slots else []}
            if self.plans is not None:
                from .ps_device import spec_for
                spec.update(spec_for(self.space, self.plans[k], names))
            vals = (torch.cat([self.params[i].detach().float().reshape(-1).cpu() for i in idx])
                    if idx else torch.zeros(0))
            dist.send(_hdr(OP_INIT, dist.get_rank(), vals.numel()), rank, group=self.group)
            _send_bytes(json.dumps(spec).encode(), rank, self.group)
            dist.send(vals, rank, group=self.group)
            for sname in spec["slot_values"]:
                sv = (torch.cat([slots[sname][i].detach().float().reshape(-1).cpu() for i in idx])
                      if idx else torch.zeros(0))
                dist.send(sv, rank, group=self.group)

    @comm_call
    def wait_ready(self, params, timeout_s=None):
        """Non-chief: block until the chief initialised every PS shard (TF WorkerSessionCreator).
        ``timeout_s`` bounds the wait (recovery: ``DTF_RECOVERY_TIMEOUT_S``) with an error that
        says which shard never became ready."""
        import datetime
        self._layout(params)
        for rank in self.ps_ranks:
            dist.send(_hdr(OP_WAIT_READY, dist.get_rank()), rank, group=self.group)
        descs = []
        for k, rank in enumerate(self.ps_ranks):
            r = torch.zeros(HDR, dtype=torch.int64)
            if timeout_s is None:
                dist.recv(r, rank, group=self.group)
            else:
                try:
                    dist.irecv(r, rank, group=self.group).wait(
                        datetime.timedelta(seconds=float(timeout_s)))
                except RuntimeError as e:
                    if "Timed out" not in str(e):
                        raise
                    raise TimeoutError(f"parameter server {k} (rank {rank}) was not initialised "
                                       f"by the chief within {float(timeout_s):.0f} s") from e
            self.global_step = max(self.global_step, int(r[1]))
            descs.append(json.loads(_recv_bytes(rank, self.group).decode()) if int(r[2]) else None)
        if all(d is not None for d in descs) and descs:
            from .ps_device import PSLink
            me = dist.get_rank()
            self.links = [PSLink(d, self.plans[k], d["workers"].index(me), self.space.device, k)
                          for k, d in enumerate(descs)]

    @comm_call
    def pull(self):
        if self.links:
            for link in self.links:
                link.pull(self.space)
            self.global_step = self.links[0].global_step
            return self.global_step
        for k, rank in enumerate(self.ps_ranks):
            dist.send(_hdr(OP_PULL, dist.get_rank()), rank, group=self.group)
        for k, rank in enumerate(self.ps_ranks):
            r = torch.zeros(HDR, dtype=torch.int64)
            dist.recv(r, rank, group=self.group)
            if k == 0:
                self.global_step = int(r[0])
            vals = torch.zeros(int(r[1]), dtype=torch.float32)
            dist.recv(vals, rank, group=self.group)
            self._assign(k, vals)
        return self.global_step

    @comm_call
    def push(self, grads=None, pull=True):
        """Send gradients (default: ``p.grad``) computed at ``self.global_step``; with
        ``pull`` the reply carries the updated shard values, copied into the local variables
        (push + pull in one round trip).  Returns the new global step."""
        if self.links:
            import time

            from .ps_device import sync_device
            t0 = time.perf_counter()
            for link in self.links:                  # gradients straight into the mailboxes
                link.copy_grads(self.space)
            sync_device(self.space.device)
            t1 = time.perf_counter()
            for link in self.links:
                link.post(self.global_step)
            steps = [link.wait() for link in self.links]
            self.global_step = steps[0]
            t2 = time.perf_counter()
            if pull:
                for link in self.links:
                    link.pull(self.space)
            t3 = time.perf_counter()
            tm = self.timing
            tm["copy_sync_ms"].append((t1 - t0) * 1e3)
            tm["wait_ms"].append((t2 - t1) * 1e3)
            tm["pull_ms"].append((t3 - t2) * 1e3)
            return self.global_step
        grads = grads or [p.grad for p in self.params]
        for k, rank in enumerate(self.ps_ranks):
            idx = self.by_ps[k]
            flat = (torch.cat([grads[i].detach().float().reshape(-1).cpu() for i in idx])
                    if idx else torch.zeros(0))
            dist.send(_hdr(OP_PUSH, dist.get_rank(), self.global_step, 1 if k == 0 else 0,
                           1 if pull else 0), rank, group=self.group)
            dist.send(flat, rank, group=self.group)
        for k, rank in enumerate(self.ps_ranks):
            r = torch.zeros(HDR, dtype=torch.int64)
            dist.recv(r, rank, group=self.group)
            if k == 0:
                self.global_step = int(r[0])
            if pull:
                vals = torch.zeros(int(r[1]), dtype=torch.float32)
                dist.recv(vals, rank, group=self.group)
                self._assign(k, vals)
        return self.global_step

    def _assign(self, k, vals):
        off = 0
        with torch.no_grad():
            for i in self.by_ps[k]:
                p = self.params[i]
                n = p.numel()
                p.copy_(vals[off:off + n].view(p.shape).to(p.device, p.dtype))
                off += n
                s = getattr(p, "_dtf_shadow", None)
                if s is not None:
                    s.copy_(p.detach())

    @comm_call
    def get_global_step(self):
        if self.links:
            self.global_step = self.links[0].global_step
            return self.global_step
        dist.send(_hdr(OP_GET_STEP, dist.get_rank()), self.ps_ranks[0], group=self.group)
        r = torch.zeros(HDR, dtype=torch.int64)
        dist.recv(r, self.ps_ranks[0], group=self.group)
        self.global_step = int(r[0])
        return self.global_step

    @comm_call
    def get_state(self):
        """(global_step, {name: tensor}, {slot_name: {name: tensor}}) across all shards."""
        values, slots, gstep = {}, {}, 0
        for k, rank in enumerate(self.ps_ranks):
            dist.send(_hdr(OP_GET_STATE, dist.get_rank()), rank, group=self.group)
            st = json.loads(_recv_bytes(rank, self.group).decode())
            if k == 0:
                gstep = st["global_step"]
            n = sum(_prod(s) for s in st["shapes"])
            flat = torch.zeros(n, dtype=torch.float32)
            dist.recv(flat, rank, group=self.group)
            for name, t in zip(st["names"], _split(flat, [tuple(s) for s in st["shapes"]])):
                values[name] = t.clone()
            for sname in st["slots"]:
                sf = torch.zeros(n, dtype=torch.float32)
                dist.recv(sf, rank, group=self.group)
                for name, t in zip(st["names"], _split(sf, [tuple(s) for s in st["shapes"]])):
                    slots.setdefault(sname, {})[name] = t.clone()
        return gstep, values, slots

    @comm_call
    def set_state(self, global_step):
        """Push the local parameter values to the PS (restore from checkpoint)."""
        for k, rank in enumerate(self.ps_ranks):
            idx = self.by_ps[k]
            flat = (torch.cat([self.params[i].detach().float().reshape(-1).cpu() for i in idx])
                    if idx else torch.zeros(0))
            dist.send(_hdr(OP_SET_STATE, dist.get_rank(), global_step), rank, group=self.group)
            dist.send(flat, rank, group=self.group)
        self.global_step = global_step

    def stop(self):
        for rank in self.ps_ranks:
            dist.send(_hdr(OP_STOP, dist.get_rank()), rank, group=self.group)

    def shutdown_ps(self):
        for rank in self.ps_ranks:
            dist.send(_hdr(OP_SHUTDOWN, dist.get_rank()), rank, group=self.group)


def _prod(s):
    n = 1
    for d in s:
        n *= d
    return n
