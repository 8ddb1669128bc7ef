"""``global_step``: the int64 step counter of TF1 (``tf.train.get_or_create_global_step``,
``run_mnist_distributed.py:114``; explicit ``tf.Variable(0, name="global_step")`` in
``templates/00_mnist_replica.py:138``).

Here it is a small object holding an int64 tensor (checkpointed as ``global_step``) plus a host
mirror so hooks (StopAtStepHook) can read it without a device sync.  In async parameter-server
mode the authoritative value lives with the PS service (``parallel/ps_service.py`` / ``ps_device.py``) and
``assign()`` syncs the local mirror.
"""
from __future__ import annotations

import threading

import torch

_default = None
_lock = threading.Lock()


class GlobalStep:
    def __init__(self, value=0, name="global_step"):
        self.name = name
        self._host = int(value)
        self.tensor = torch.tensor(int(value), dtype=torch.int64)
        self.tensor._dtf_name = name

    def value(self) -> int:
        return self._host

    def __int__(self):
        return self._host

    def assign(self, v: int):
        self._host = int(v)
        self.tensor.fill_(int(v))

    def assign_add(self, d: int = 1) -> int:
        with _lock:
            self._host += int(d)
            self.tensor.fill_(self._host)
            return self._host

    def __repr__(self):
        return f"<GlobalStep {self._host}>"


def get_or_create_global_step() -> GlobalStep:
    global _default
    if _default is None:
        _default = GlobalStep()
    return _default


def get_global_step():
    return _default


def reset_global_step():
    global _default
    _default = None


def create_global_step(value=0) -> GlobalStep:
    global _default
    _default = GlobalStep(value)
    return _default


def increment(gs, by: int = 1) -> int:
    if isinstance(gs, GlobalStep):
        return gs.assign_add(by)
    if isinstance(gs, torch.Tensor):
        gs.add_(by)
        return int(gs.item())
    raise TypeError(type(gs))
