"""Launcher-hosted rendezvous store and cluster epochs (failure recovery).

The reference relies on TF1's ``MonitoredTrainingSession`` recreating its session after a task
of the cluster died (``/root/reference/run_mnist_distributed.py:128-132,146``) and on the
Supervisor's non-chiefs retrying every ``recovery_wait_secs`` (``templates/00_mnist_replica.py:
196-204``).  Here every task is one process of a torch.distributed world, so a death breaks the
world; recovery means forming a NEW world with the restarted task.

* The rendezvous TCPStore is hosted by the LAUNCHER (``cluster/launcher.py``), never by a task:
  the chief can die and be restarted like any other task.  Tasks find it through
  ``DTF_STORE_ADDR=host:port``.
* The store holds the cluster EPOCH (``dtf/epoch``).  Before it restarts a crashed task the
  launcher bumps the epoch; every process group is created under ``PrefixStore("g<epoch>")``.
  A restarted task simply joins the current epoch; a surviving task notices the bump (an
  :class:`EpochWatcher` thread polls the store, and its own collectives fail on the dead peer),
  tears down its group and joins the new epoch -- so all of them meet there without any extra
  coordination, however many tasks died.
* Recovery is attempted only when a launcher that restarts tasks is present
  (``DTF_MAX_RESTARTS`` > 0): otherwise a dead peer is a plain error, as it should be.
"""
from __future__ import annotations

import datetime
import os
import threading
import time

import torch.distributed as dist

EPOCH_KEY = "dtf/epoch"


class ClusterChanged(ConnectionError):
    """A task of the cluster died and the launcher restarted it: this process must leave its
    process group and join the new epoch (MonitoredTrainingSession recovers from it)."""


def store_address():
    a = os.environ.get("DTF_STORE_ADDR", "")
    if not a:
        return None
    host, _, port = a.rpartition(":")
    return host, int(port)


def recovery_enabled():
    return store_address() is not None and int(os.environ.get("DTF_MAX_RESTARTS", "0") or 0) > 0


def connect(timeout_s=600, host=None, port=None, is_master=False):
    """The cluster store: the launcher's (``DTF_STORE_ADDR``) when present, else a store at
    ``host:port`` (hosted by this process when ``is_master``: the chief of a hand-started
    cluster, the reference's own deployment)."""
    addr = store_address()
    if addr is not None:
        host, port, is_master = addr[0], addr[1], False
    return dist.TCPStore(host, port, None, is_master,
                         timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)


def current_epoch(store):
    return int(store.add(EPOCH_KEY, 0))


def bump_epoch(store):
    return int(store.add(EPOCH_KEY, 1))


def recovery_timeout_s(default=120.0):
    """Bound of every wait on the recovery path (the launcher's epoch bump, the other tasks
    joining the new epoch, the chief re-seeding the parameter servers): ``DTF_RECOVERY_TIMEOUT_S``
    (default 120 s).  Tests set it below their own budget so a stalled wait names itself."""
    return float(os.environ.get("DTF_RECOVERY_TIMEOUT_S", "") or default)


def arrive(store, epoch, rank, world_size, timeout_s, what="join"):
    """Bounded arrival barrier of cluster epoch ``epoch`` before its process group is created:
    the group's own rendezvous would wait out the store timeout (minutes) for a task that never
    comes; this fails after ``timeout_s`` naming the ranks that did not arrive."""
    store.set(f"g{epoch}/arrived/{rank}", "1")
    store.add(f"g{epoch}/arrived_n", 1)
    t0 = time.time()
    while int(store.add(f"g{epoch}/arrived_n", 0)) < world_size:
        if time.time() - t0 > timeout_s:
            missing = [r for r in range(world_size)
                       if not store.check([f"g{epoch}/arrived/{r}"])]
            raise TimeoutError(f"{what}: waited {timeout_s:.0f} s for rank(s) {missing} of "
                               f"{world_size} to join cluster epoch {epoch}")
        time.sleep(0.02)


def wait_for_epoch_after(store, epoch, timeout_s=120.0):
    """Block until the launcher moved the cluster past ``epoch`` (it bumps before restarting a
    task); bounded, so a peer death that nobody restarts fails instead of hanging."""
    t0 = time.time()
    while True:
        e = current_epoch(store)
        if e > epoch:
            return e
        if time.time() - t0 > timeout_s:
            raise TimeoutError(f"cluster epoch stayed at {epoch} for {timeout_s:.0f} s: the "
                               f"failed task was not restarted")
        time.sleep(0.05)


class EpochWatcher:
    """Polls the cluster epoch in the background (its own store connection, so it never blocks
    behind this process's collectives); ``changed`` turns True once the launcher bumped it."""

    def __init__(self, epoch, interval_s=0.2):
        self.epoch = epoch
        self.interval_s = interval_s
        self._changed = threading.Event()
        self._stop = threading.Event()
        self._thread = None

    def start(self):
        if store_address() is None:
            return self
        self._thread = threading.Thread(target=self._run, name="dtf-epoch-watch", daemon=True)
        self._thread.start()
        return self

    def _run(self):
        try:
            store = connect(timeout_s=30)
        except Exception:
            return
        while not self._stop.wait(self.interval_s):
            try:
                if current_epoch(store) > self.epoch:
                    self._changed.set()
                    return
            except Exception:      # launcher gone: the job is ending
                return

    @property
    def changed(self):
        return self._changed.is_set()

    def stop(self):
        self._stop.set()


def init_group(backend, rank, world_size, store, epoch, timeout_s=600, **kw):
    """A process group of this epoch (``PrefixStore("g<epoch>")`` over the cluster store)."""
    dist.init_process_group(backend, store=dist.PrefixStore(f"g{epoch}", store), rank=rank,
                            world_size=world_size,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)


def leave_group():
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:          # the group may already be broken
            pass
