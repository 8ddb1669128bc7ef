"""Step-phase timing and trace annotations (SURVEY.md §5.1 "New": HIP-event step-phase timers,
roctx ranges; the reference only had wall-clock ``logger.ProfileKV``).

* :class:`StepTimer` — HIP events recorded on the current stream at phase boundaries
  (``forward``/``backward``/``comm``/``optimizer`` by default, any name allowed); elapsed times
  are read only when :meth:`StepTimer.summary` is called, so timing adds no host sync to the step.
  The Optimizer records ``backward`` / ``comm`` / ``optimizer`` automatically while a timer is
  :func:`enable`-d; wrap the model call in ``timer.phase("forward")``.
* :func:`range` — a roctx range (``libroctx64.so``) visible in ``rocprofv3 --marker-trace``; a
  no-op when the library is absent.  Also pushed automatically around each timed phase.

    timer = dtf.profiler.enable()
    with timer.phase("forward"):
        loss = loss_fn(model(x), y)
    opt.minimize(loss)
    print(timer.summary())      # {'forward': ms, 'backward': ms, 'comm': ms, 'optimizer': ms}
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import time
from collections import defaultdict

import torch

_roctx = None
_roctx_tried = False


def _lib():
    global _roctx, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        for name in ("libroctx64.so", "libroctx64.so.4", ctypes.util.find_library("roctx64")):
            if not name:
                continue
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx / nvtx naming
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


class StepTimer:
    def __init__(self, device=None):
        self.cuda = torch.cuda.is_available() if device is None else torch.device(device).type == "cuda"
        self._pending = []            # (name, start, end)
        self.totals = defaultdict(float)
        self.counts = defaultdict(int)

    def _event(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    @contextlib.contextmanager
    def phase(self, name: str):
        start = self._event()
        with range(name):
            try:
                yield
            finally:
                self._pending.append((name, start, self._event()))

    def _drain(self):
        if self.cuda and self._pending:
            self._pending[-1][2].synchronize()
        for name, s, e in self._pending:
            ms = s.elapsed_time(e) if self.cuda else (e - s) * 1e3
            self.totals[name] += ms
            self.counts[name] += 1
        self._pending.clear()

    def summary(self, reset=True):
        """Average milliseconds per occurrence of each phase since the last reset."""
        self._drain()
        out = {k: round(self.totals[k] / max(self.counts[k], 1), 4) for k in self.totals}
        if reset:
            self.totals.clear()
            self.counts.clear()
        return out


_active: StepTimer | None = None


def enable(device=None) -> StepTimer:
    global _active
    _active = StepTimer(device)
    return _active


def disable():
    global _active
    _active = None


def active() -> StepTimer | None:
    return _active


@contextlib.contextmanager
def maybe_phase(name: str):
    """Used by the framework internals: times ``name`` only when a timer is enabled."""
    t = _active
    if t is None:
        yield
    else:
        with t.phase(name):
            yield
