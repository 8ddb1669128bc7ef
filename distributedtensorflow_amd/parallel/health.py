"""Replica consistency checks and peer failure detection (SURVEY.md §5.2 / §5.3 "New").

* :func:`check_replicas_consistent` — synchronous data parallelism must keep every replica's
  variables BIT-identical (same all-reduced gradient, same fused update).  Each rank hashes its
  flat master buffer (a position-weighted integer fingerprint of the raw bits, so a single
  flipped bit anywhere changes it), the fingerprints are all-gathered and compared.
  :class:`ReplicaConsistencyHook` runs it every N steps inside a MonitoredTrainingSession.
* :class:`Heartbeat` — every rank writes ``hb/<rank>`` = wall time into the job's TCPStore from a
  daemon thread and watches its peers; a peer silent for ``timeout_s`` is reported in
  ``failed_peers`` and :class:`HeartbeatHook` turns that into a ``ConnectionError`` — one of
  MonitoredTrainingSession's recoverable errors, so the session restores from the latest
  checkpoint instead of hanging in a collective (the RCCL watchdog, enabled by
  ``init_process_group_from_env``, aborts communicators stuck past the PG timeout).
"""
from __future__ import annotations

import os
import threading
import time

import torch
import torch.distributed as dist

from ..train.hooks import SessionRunHook


class ReplicaDivergence(RuntimeError):
    pass


def fingerprint(t: torch.Tensor) -> int:
    """64-bit position-weighted fingerprint of a tensor's raw bits (device-side, one sync)."""
    flat = t.detach().contiguous().reshape(-1)
    if flat.element_size() == 4:
        bits = flat.view(torch.int32).to(torch.int64)
    elif flat.element_size() == 2:
        bits = flat.view(torch.int16).to(torch.int64)
    elif flat.element_size() == 8:
        bits = flat.view(torch.int64)
    else:
        bits = flat.view(torch.uint8).to(torch.int64)
    w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    return int((bits * w).sum().item())


def check_replicas_consistent(tensors, group=None, raise_on_mismatch=True):
    """``tensors``: a tensor, a list of tensors, or an object with a ``master`` buffer (FlatSpace)
    / a ``space`` (Optimizer).  Returns the list of per-rank fingerprints."""
    if hasattr(tensors, "space") and tensors.space is not None:
        if hasattr(tensors, "synchronize_variables"):
            tensors.synchronize_variables()      # pending overlapped variable gathers
        tensors = tensors.space.master
    elif hasattr(tensors, "master"):
        tensors = tensors.master
    if isinstance(tensors, torch.Tensor):
        tensors = [tensors]
    fp = [fingerprint(t) for t in tensors]
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [fp]
    gathered = [None] * dist.get_world_size(group)
    dist.all_gather_object(gathered, fp, group=group)
    if raise_on_mismatch and any(g != gathered[0] for g in gathered):
        bad = [r for r, g in enumerate(gathered) if g != gathered[0]]
        raise ReplicaDivergence(f"replica variables diverged on ranks {bad} (vs rank 0)")
    return gathered


class ReplicaConsistencyHook(SessionRunHook):
    def __init__(self, optimizer, every_n_steps=100, group=None):
        self.optimizer, self.every, self.group = optimizer, every_n_steps, group
        self.checks = 0
        self._n = 0

    def after_run(self, run_context, run_values):
        self._n += 1
        if self._n % self.every == 0:
            check_replicas_consistent(self.optimizer, self.group)
            self.checks += 1


class Heartbeat:
    def __init__(self, rank=None, world_size=None, interval_s=1.0, timeout_s=30.0, store=None,
                 prefix="hb"):
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world_size is None else world_size
        self.interval, self.timeout, self.prefix = interval_s, timeout_s, prefix
        if store is None:
            store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"),
                                  int(os.environ["MASTER_PORT"]), is_master=False,
                                  timeout=__import__("datetime").timedelta(seconds=60))
        self.store = store
        self.failed_peers: set[int] = set()
        self._stop = threading.Event()
        self._start = time.time()
        self._thread = threading.Thread(target=self._run, daemon=True, name="dtf-heartbeat")

    def start(self):
        self._beat()
        self._thread.start()
        return self

    def _beat(self):
        self.store.set(f"{self.prefix}/{self.rank}", repr(time.time()))

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self._beat()
                now = time.time()
                for r in range(self.world):
                    if r == self.rank:
                        continue
                    key = f"{self.prefix}/{r}"
                    if not self.store.check([key]):
                        if now - self._start > self.timeout:
                            self.failed_peers.add(r)
                        continue
                    last = float(self.store.get(key).decode())
                    if now - last > self.timeout:
                        self.failed_peers.add(r)
                    else:
                        self.failed_peers.discard(r)
            except Exception:          # store gone = the job is shutting down / master died
                self.failed_peers.add(-1)

    def stop(self):
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(timeout=2 * self.interval)


class HeartbeatHook(SessionRunHook):
    def __init__(self, heartbeat: Heartbeat):
        self.hb = heartbeat

    def before_run(self, run_context):
        if self.hb.failed_peers:
            raise ConnectionError(f"heartbeat lost from peers {sorted(self.hb.failed_peers)}")

    def end(self, session):
        self.hb.stop()
