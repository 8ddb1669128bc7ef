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

import itertools
import os

import torch
import torch.distributed as dist

_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
_DTYPES = {torch.float32: 7, torch.bfloat16: 9, torch.float16: 6, torch.int64: 4,
           torch.int32: 2, torch.uint8: 1}
_COUNTER = itertools.count()


class C10dComm:
    """torch.distributed collectives (async_op=True) on a process group."""

    kind = "c10d"

    def __init__(self, group=None):
        self.group = group

    def all_reduce(self, t):
        return dist.all_reduce(t, group=self.group, async_op=True)

    def reduce_scatter(self, out, inp):
        return dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=True)

    def all_gather(self, out, inp):
        return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)

    def reduce(self, t, dst):
        return dist.reduce(t, dst=dst, group=self.group, async_op=True)

    def broadcast(self, t, src):
        return dist.broadcast(t, src=src, group=self.group, async_op=True)

    def close(self, abort=False):
        pass


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
        key = f"dtf/rccl_uid/{next(_COUNTER)}"
        if self.rank == 0:
            uid = self.K.rccl_unique_id()
            store.set(key, uid)
        else:
            uid = bytes(store.get(key))
        self.comm = self.K.rccl_comm_init(uid, self.world, self.rank, self.device.index)
        # highest priority: the collectives should not queue behind compute kernels
        self.stream = torch.cuda.Stream(self.device, priority=-1)

    def _issue(self, fn, *tensors):
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)            # the producers of the operands ran before issue
        fn(self.stream.cuda_stream)
        for t in tensors:
            t.record_stream(self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _Done(ev)

    @staticmethod
    def _dt(t):
        try:
            return _DTYPES[t.dtype]
        except KeyError:
            raise TypeError(f"rccl: unsupported dtype {t.dtype}") from None

    def all_reduce(self, t, op="sum"):
        return self._issue(lambda s: self.K.rccl_all_reduce(
            self.comm, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), _OPS[op], s), t)

    def reduce_scatter(self, out, inp, op="sum"):
        if inp.numel() != out.numel() * self.world:
            raise ValueError("rccl reduce_scatter: input must be world x output")
        return self._issue(lambda s: self.K.rccl_reduce_scatter(
            self.comm, inp.data_ptr(), out.data_ptr(), out.numel(), self._dt(out), _OPS[op], s),
            out, inp)

    def all_gather(self, out, inp):
        if out.numel() != inp.numel() * self.world:
            raise ValueError("rccl all_gather: output must be world x input")
        return self._issue(lambda s: self.K.rccl_all_gather(
            self.comm, inp.data_ptr(), out.data_ptr(), inp.numel(), self._dt(inp), s), out, inp)

    def reduce(self, t, dst, op="sum"):
        return self._issue(lambda s: self.K.rccl_reduce(
            self.comm, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), _OPS[op], dst, s), t)

    def broadcast(self, t, src):
        return self._issue(lambda s: self.K.rccl_broadcast(
            self.comm, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), src, s), t)

    def async_error(self):
        return self.K.rccl_async_error(self.comm)

    def close(self, abort=False):
        if self.comm:
            if not abort:
                self.stream.synchronize()
            self.K.rccl_comm_destroy(self.comm, int(abort))
            self.comm = 0


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
