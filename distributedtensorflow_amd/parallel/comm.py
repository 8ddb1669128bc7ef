"""Communicators used by the gradient reducers: torch.distributed (c10d) or native RCCL.

SURVEY.md §5.8 plans the data plane as "a C++ wrapper over rccl.h ... collectives enqueued on a
dedicated comm HIP stream, ordered against the compute stream by hipEvents".  Both
implementations below expose the same five asynchronous collectives on flat-buffer views and
return a handle whose ``wait()`` makes the CURRENT (compute) stream wait for the collective --
never the host:

* :class:`C10dComm` -- ``torch.distributed`` (ProcessGroupNCCL = RCCL on ROCm; gloo on CPU),
  the default;
* :class:`RcclComm` -- ``csrc/kernels/rccl_comm.cpp``: an ``ncclComm_t`` created with
  ``ncclCommInitRank`` (unique id exchanged through the rendezvous TCPStore), every collective
  enqueued on ONE high-priority comm stream behind an event recorded on the compute stream at
  issue, completion handed back as an event.  No c10d work objects or watchdog thread on the
  gradient path.  Selected with ``DTF_COMM=rccl`` (or ``comm="rccl"`` on the strategies).
"""
from __future__ import annotations

import os
import threading
import time

import torch
import torch.distributed as dist

_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
_DTYPES = {torch.float32: 7, torch.bfloat16: 9, torch.float16: 6, torch.int64: 4,
           torch.int32: 2, torch.uint8: 1}
# RCCL unique-id store keys: "dtf/rccl_uid/<n>" under the process group's store, which the
# launcher scopes per cluster epoch (PrefixStore "g<epoch>").  ``n`` counts communicators created
# in THIS world and restarts at 0 whenever a world is formed (reset_uid_index, called by
# init_process_group_from_env): a restarted rank and the survivors then agree on the key.
_uid_index = 0


def reset_uid_index():
    global _uid_index
    _uid_index = 0


def _next_uid_key():
    global _uid_index
    k = f"dtf/rccl_uid/{_uid_index}"
    _uid_index += 1
    return k


def _watchdog():
    from .watchdog import get_watchdog
    return get_watchdog()


class C10dComm:
    """torch.distributed collectives (async_op=True) on a process group."""

    kind = "c10d"

    def __init__(self, group=None):
        self.group = group
        self.wd = _watchdog()
        self._nccl = dist.get_backend(group) == "nccl"
        self._aborted = False
        self.wd.add_abort(self.abort)

    def _track(self, work, what):
        self.wd.watch(work.is_completed, f"c10d {what}")
        return work

    def all_reduce(self, t):
        self.wd.check()
        return self._track(dist.all_reduce(t, group=self.group, async_op=True), "all_reduce")

    def reduce_scatter(self, out, inp):
        self.wd.check()
        return self._track(dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=True),
                           "reduce_scatter")

    def all_gather(self, out, inp):
        self.wd.check()
        return self._track(dist.all_gather_into_tensor(out, inp, group=self.group,
                                                       async_op=True), "all_gather")

    def reduce(self, t, dst):
        self.wd.check()
        return self._track(dist.reduce(t, dst=dst, group=self.group, async_op=True), "reduce")

    def broadcast(self, t, src):
        self.wd.check()
        return self._track(dist.broadcast(t, src=src, group=self.group, async_op=True),
                           "broadcast")

    def abort(self):
        """Watchdog trip: abort the RCCL communicators of the process group, so kernels blocked
        on a dead peer exit (gloo has no device-side wait to break; its own timeout applies)."""
        if self._aborted or not self._nccl:
            return
        self._aborted = True
        abort = getattr(dist.distributed_c10d, "_abort_process_group", None)
        if abort is not None and dist.is_initialized():
            abort(self.group) if self.group is not None else abort()

    def close(self, abort=False):
        """``abort``: the world broke (recovery) -- abort the process group's communicators
        BEFORE leaving it, so nothing stays blocked on the dead peer; the watchdog callback is
        unregistered only afterwards (a later trip could otherwise no longer reach it)."""
        if abort:
            self.abort()
        self.wd.remove_abort(self.abort)


class _Done:
    """Completion of a native collective: an event on the comm stream."""

    __slots__ = ("ev",)

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)

    def is_completed(self):
        return self.ev.query()


def torch_rccl_path():
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


class RcclComm:
    """A native RCCL communicator over the ranks of ``group`` (see module docstring)."""

    kind = "rccl"

    def __init__(self, group=None, device=None, store=None):
        from ..ops import native
        self.K = native.kernels()
        self.version = self.K.rccl_load(torch_rccl_path())
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        store = store or dist.distributed_c10d._get_default_store()
        key = _next_uid_key()
        if self.rank == 0:
            uid = self.K.rccl_unique_id()
            store.set(key, uid)
        else:
            uid = bytes(store.get(key))
        self.comm = self.K.rccl_comm_init(uid, self.world, self.rank, self.device.index)
        # highest priority: the collectives should not queue behind compute kernels
        self.stream = torch.cuda.Stream(self.device, priority=-1)
        # bounded waits: ncclCommAbort from the watchdog on a deadline / async error / epoch bump.
        # The lock guards the handle and the in-flight enqueue count only, and is never held
        # across a call into RCCL that can block: the communicator is a blocking one, so an
        # enqueue may wait inside RCCL on a dead peer (lazy connection set-up), and the watchdog
        # thread must still be able to probe it and abort it then
        self._lock = threading.Lock()
        self._inuse = 0
        self.wd = _watchdog()
        self.wd.add_abort(self.abort)
        self.wd.add_probe(self._probe)

    def _probe(self):
        # ncclCommGetAsyncError never blocks and is safe beside an in-flight enqueue; the lock
        # only keeps abort / close from releasing the handle during the call
        with self._lock:
            if not self.comm:
                return None
            r = self.K.rccl_async_error(self.comm)
        return f"rccl async error {r}" if r not in (0, 7) else None    # 7 = ncclInProgress

    def _enqueue(self, fn, stream, what):
        """Run ``fn(comm, stream)`` (one RCCL enqueue) with the handle pinned by the in-flight
        count, not by the lock.  The collective's deadline is registered BEFORE the call, so an
        enqueue that blocks inside RCCL trips the watchdog like a kernel that never completes;
        returns the completion cell the caller fills with the collective's event."""
        from .strategy import CommError
        cell = []
        self.wd.watch(lambda: bool(cell) and cell[0](), f"rccl {what}")
        with self._lock:
            comm = self.comm
            if not comm:
                cell.append(lambda: True)
                raise CommError("rccl communicator was aborted")
            self._inuse += 1
        try:
            fn(comm, stream)
        except BaseException:
            cell.append(lambda: True)        # the error is the caller's to report
            raise
        finally:
            with self._lock:
                self._inuse -= 1
                aborted = not self.comm
        if aborted:
            cell.append(lambda: True)
            raise CommError(f"rccl communicator was aborted during the {what} enqueue")
        return cell

    def _issue(self, fn, *tensors, what="collective"):
        """Enqueue ``fn(comm, stream)`` on the comm stream, ordered after the caller's stream."""
        self.wd.check()
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)            # the producers of the operands ran before issue
        cell = self._enqueue(fn, self.stream.cuda_stream, what)
        for t in tensors:
            t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        cell.append(ev.query)
        return _Done(ev)

    @staticmethod
    def _dt(t):
        try:
            return _DTYPES[t.dtype]
        except KeyError:
            raise TypeError(f"rccl: unsupported dtype {t.dtype}") from None

    def all_reduce(self, t, op="sum"):
        return self._issue(lambda c, s: self.K.rccl_all_reduce(
            c, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), _OPS[op], s), t,
            what="all_reduce")

    @staticmethod
    def _overlap(a, b):
        ea, eb = a.element_size(), b.element_size()
        return a.data_ptr() < b.data_ptr() + b.numel() * eb and \
            b.data_ptr() < a.data_ptr() + a.numel() * ea

    def reduce_scatter(self, out, inp, op="sum"):
        if inp.numel() != out.numel() * self.world:
            raise ValueError("rccl reduce_scatter: input must be world x output")
        # NCCL's in-place rule: an output inside the input must be exactly this rank's chunk
        # (recvbuff == sendbuff + rank * recvcount); any other overlap is undefined behaviour
        # that a world-1 run can never show (the colocated PS reduces in place)
        if self._overlap(out, inp) and out.data_ptr() != \
                inp.data_ptr() + self.rank * out.numel() * out.element_size():
            raise ValueError("rccl reduce_scatter: in-place output must be the input's chunk "
                             f"{self.rank} (recvbuff == sendbuff + rank * count)")
        return self._issue(lambda c, s: self.K.rccl_reduce_scatter(
            c, inp.data_ptr(), out.data_ptr(), out.numel(), self._dt(out), _OPS[op], s),
            out, inp, what="reduce_scatter")

    def all_gather(self, out, inp):
        if out.numel() != inp.numel() * self.world:
            raise ValueError("rccl all_gather: output must be world x input")
        if self._overlap(out, inp) and inp.data_ptr() != \
                out.data_ptr() + self.rank * inp.numel() * inp.element_size():
            raise ValueError("rccl all_gather: in-place input must be the output's chunk "
                             f"{self.rank} (sendbuff == recvbuff + rank * count)")
        return self._issue(lambda c, s: self.K.rccl_all_gather(
            c, inp.data_ptr(), out.data_ptr(), inp.numel(), self._dt(inp), s), out, inp,
            what="all_gather")

    def reduce(self, t, dst, op="sum"):
        return self._issue(lambda c, s: self.K.rccl_reduce(
            c, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), _OPS[op], dst, s), t,
            what="reduce")

    def broadcast(self, t, src):
        return self._issue(lambda c, s: self.K.rccl_broadcast(
            c, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), src, s), t,
            what="broadcast")

    def async_error(self):
        return self.K.rccl_async_error(self.comm)

    def abort(self):
        """ncclCommAbort (idempotent; never waits for an in-flight enqueue): RCCL kernels still
        spinning on a dead peer see the abort flag and exit, so the comm stream drains, and an
        enqueue blocked inside RCCL on another thread returns with an error (its caller then
        raises CommError).  The handle is unpublished first, so no new enqueue starts on it."""
        with self._lock:
            c, self.comm = self.comm, 0
        if c:
            self.K.rccl_comm_destroy(c, 1)

    def close(self, abort=False):
        self.wd.remove_abort(self.abort)
        self.wd.remove_probe(self._probe)
        if abort:
            self.abort()
            return
        with self._lock:
            c, self.comm = self.comm, 0
        if c:
            # a graceful destroy frees the communicator: let an enqueue still in RCCL on another
            # thread leave it first (bounded; a stuck one is the watchdog's, via abort)
            t0 = time.monotonic()
            while self._inuse and time.monotonic() - t0 < 30:
                time.sleep(0.001)
            self.stream.synchronize()
            self.K.rccl_comm_destroy(c, 1 if self._inuse else 0)


def make_comm(kind=None, group=None, device=None):
    """``kind``: "c10d" | "rccl" | None (``DTF_COMM``, default c10d).  Native RCCL needs a GPU
    process group (backend nccl); anything else stays on c10d."""
    kind = kind or os.environ.get("DTF_COMM", "c10d")
    if kind == "rccl":
        if not torch.cuda.is_available() or dist.get_backend(group) != "nccl":
            raise ValueError("DTF_COMM=rccl needs CUDA/HIP tensors and an nccl process group")
        return RcclComm(group, device)
    if kind != "c10d":
        raise ValueError(f"unknown communicator {kind!r} (c10d or rccl)")
    return C10dComm(group)
