"""Collective watchdog: every collective on the gradient path has a deadline.

The reference survives a preempted task because TF1's ``MonitoredTrainingSession`` recreates its
session on ``AbortedError`` / ``UnavailableError`` (``/root/reference/run_mnist_distributed.py:
128-132,146``).  On a GPU collective world the equivalent failure is silent: when a peer dies,
the survivors' RCCL kernels spin on flags the dead peer will never write, the compute stream waits
on them, and the host blocks in its next synchronisation -- forever with a native communicator,
or for the process group's timeout with c10d.

One :class:`CommWatchdog` per process (a daemon thread, 50 ms poll) makes that bounded:

* every communicator registers each collective it issues (``watch``: a completion probe and a
  deadline, ``DTF_COMM_TIMEOUT_S``, default 300 s) and an ``abort`` callback
  (``ncclCommAbort`` for the native communicator, ``_abort_process_group`` for c10d);
* extra probes report failures the collective itself cannot: the native communicator's
  ``ncclCommGetAsyncError`` and the launcher's cluster-epoch bump (a peer was restarted, so the
  current world is broken even if nothing is in flight yet);
* on the first failure the watchdog TRIPS: it runs every abort callback -- which makes the
  blocked RCCL kernels exit, so the streams and the host drain -- and records the reason.
  :meth:`check` (called by the communicators before issuing, by the reducers' ``finish`` and by
  ``MonitoredTrainingSession`` after each step) then raises :class:`CommError`, which the
  session recovers from under a restarting launcher and which ends the process loudly otherwise.
"""
from __future__ import annotations

import os
import threading
import time


def default_timeout_s():
    return float(os.environ.get("DTF_COMM_TIMEOUT_S", "300") or 300)


class CommWatchdog:
    def __init__(self, timeout_s=None, interval_s=0.05):
        self.timeout_s = default_timeout_s() if timeout_s is None else float(timeout_s)
        self.interval_s = interval_s
        self._lock = threading.Lock()
        self._inflight = []            # [done_fn, deadline, what]
        self._aborts = []              # callables, run once when tripped
        self._probes = []              # callables -> failure reason or None
        self._failed = None
        self._tripped = threading.Event()
        self._stop = threading.Event()
        self._thread = None
        self.trip_time = None

    # -- registration
    def watch(self, done_fn, what="collective"):
        """Track one in-flight collective: ``done_fn()`` turns True when it completed."""
        with self._lock:
            self._inflight.append([done_fn, time.monotonic() + self.timeout_s, what])
        self._ensure_thread()

    def add_abort(self, fn):
        with self._lock:
            self._aborts.append(fn)
        if self._tripped.is_set():    # registered after the trip: abort right away
            self._run_abort(fn)

    def remove_abort(self, fn):
        with self._lock:
            if fn in self._aborts:
                self._aborts.remove(fn)

    def add_probe(self, fn):
        with self._lock:
            self._probes.append(fn)
        self._ensure_thread()

    def remove_probe(self, fn):
        with self._lock:
            if fn in self._probes:
                self._probes.remove(fn)

    # -- state
    @property
    def failed(self):
        return self._failed

    def check(self):
        if self._failed is not None:
            from .strategy import CommError
            raise CommError(f"collective watchdog: {self._failed}")

    def inflight(self):
        with self._lock:
            return len(self._inflight)

    def trip(self, reason):
        with self._lock:
            if self._failed is not None:
                return
            self._failed = reason
            self.trip_time = time.monotonic()
            aborts = list(self._aborts)
        print(f"[dtf] collective watchdog tripped: {reason}; aborting "
              f"{len(aborts)} communicator(s)", flush=True)
        for fn in aborts:
            self._run_abort(fn)
        self._tripped.set()

    @staticmethod
    def _run_abort(fn):
        try:
            fn()
        except Exception as e:     # an abort of an already-broken communicator may itself fail
            print(f"[dtf] collective watchdog: abort failed: {type(e).__name__}: {e}", flush=True)

    def wait_tripped(self, timeout=None):
        return self._tripped.wait(timeout)

    # -- polling
    def poll_once(self):
        if self._failed is not None:
            return
        with self._lock:
            probes = list(self._probes)
            items = list(self._inflight)
        for p in probes:
            try:
                r = p()
            except Exception as e:
                r = f"probe failed: {type(e).__name__}: {e}"
            if r:
                self.trip(r)
                return
        now = time.monotonic()
        done = []
        for it in items:
            fn, deadline, what = it
            try:
                ok = fn()
            except Exception as e:     # an errored work object is a failed collective
                self.trip(f"{what}: {type(e).__name__}: {e}")
                return
            if ok:
                done.append(it)
            elif now > deadline:
                self.trip(f"{what} did not complete within {self.timeout_s:g} s "
                          f"(DTF_COMM_TIMEOUT_S): a peer is dead or hung")
                return
        if done:
            with self._lock:
                ids = {id(d) for d in done}
                self._inflight = [i for i in self._inflight if id(i) not in ids]

    def _ensure_thread(self):
        if self._thread is not None or self._stop.is_set():
            return
        with self._lock:
            if self._thread is not None:
                return
            self._thread = threading.Thread(target=self._run, name="dtf-comm-watchdog",
                                            daemon=True)
            self._thread.start()

    def _run(self):
        while not self._stop.wait(self.interval_s):
            self.poll_once()
            if self._failed is not None:
                return

    def stop(self):
        self._stop.set()


_watchdog = None
_wd_lock = threading.Lock()


def get_watchdog():
    """The process's watchdog for the CURRENT world (replaced by :func:`reset_watchdog` when a
    recovered world is formed)."""
    global _watchdog
    with _wd_lock:
        if _watchdog is None:
            _watchdog = CommWatchdog()
        return _watchdog


def reset_watchdog():
    """A new world was formed (recovery): stop the old watchdog (its communicators are gone) and
    start clean."""
    global _watchdog
    with _wd_lock:
        if _watchdog is not None:
            _watchdog.stop()
        _watchdog = CommWatchdog()
        return _watchdog


def check():
    """Raise :class:`CommError` when the current world's watchdog tripped (cheap: one load)."""
    w = _watchdog
    if w is not None and w._failed is not None:
        w.check()


__all__ = ["CommWatchdog", "get_watchdog", "reset_watchdog", "check", "default_timeout_s"]
