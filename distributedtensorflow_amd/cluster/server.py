"""Per-task server: ``tf.train.Server(cluster, job_name, task_index)`` semantics.

Reference: ``run_mnist_distributed.py:95-104`` / ``templates/00_mnist_replica.py:113-118``
(SURVEY R5).  Every task of the cluster (chief/worker/ps) is one OS process; constructing the
Server joins it into a single torch.distributed world whose TCPStore rendezvous is hosted by the
chief's ``host:port`` (rank 0).  The ``gloo`` default group carries the parameter-server
protocol (any-source receives); GPU workers additionally get an RCCL group among themselves
(``worker_group``) for collective data parallelism.

``join()`` on a ``ps`` task runs the parameter-server service and RETURNS cleanly when all
workers are done, on SIGINT/SIGTERM or on the chief's shutdown request (the reference's PS never
exits: ``README.md:7`` TODO).

Recovery (TF's ``_RecoverableSession`` recreating the session after a task of the cluster died,
reference ``run_mnist_distributed.py:146``): see :mod:`.rendezvous`.  Under the
launcher the rendezvous TCPStore lives in the launcher process, so ANY task -- the chief
included -- can die and be restarted; every process group is created for the cluster EPOCH the
launcher bumps before each restart, and :meth:`restart_group` moves a surviving task to it.
Hand-started clusters (the reference's deployment) keep the chief-hosted store and fail fast.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import rendezvous
from .spec import ClusterSpec, Config


class Server:
    def __init__(self, cluster, job_name, task_index=0, config=None, start=True,
                 protocol="dtf", worker_backend=None, timeout_s=600, ps_device="cpu"):
        if isinstance(cluster, Config):
            cluster = cluster.cluster_spec()
        self.cluster = ClusterSpec(cluster)
        self.job_name = job_name
        self.task_index = int(task_index)
        self.config = config
        self.protocol = protocol
        self.rank = self.cluster.rank_of(job_name, self.task_index)
        self.world_size = self.cluster.world_size()
        self.host, self.port = self.cluster.rendezvous_address()
        self.worker_backend = worker_backend
        self.timeout_s = timeout_s
        self.ps_device = ps_device
        self.worker_group = None
        self.store = None
        self.generation = -1
        self.watcher = None
        self._started = False
        if start:
            self.start()

    # -- TF API
    @property
    def target(self) -> str:
        return f"{self.protocol}://{self.host}:{self.port}"

    @property
    def server_def(self):
        return {"cluster": self.cluster.as_dict(), "job_name": self.job_name,
                "task_index": self.task_index}

    def worker_ranks(self):
        out = [self.cluster.rank_of("chief", 0)] if self.cluster.num_tasks("chief") else []
        out += [self.cluster.rank_of("worker", i) for i in range(self.cluster.num_tasks("worker"))]
        return out

    def ps_ranks(self):
        return [self.cluster.rank_of("ps", i) for i in range(self.cluster.num_tasks("ps"))]

    @property
    def is_chief(self):
        return (self.job_name, self.task_index) == self.cluster.chief()

    def start(self):
        if self._started:
            return
        if not dist.is_initialized():
            if self.store is None:
                # the launcher's store (DTF_STORE_ADDR); without a launcher the chief hosts it
                self.store = rendezvous.connect(self.timeout_s, self.host, self.port,
                                                is_master=self.rank == 0)
            self.generation = rendezvous.current_epoch(self.store)
            if rendezvous.store_address() is not None:
                # launcher-hosted store: bounded arrival barrier first, so a task that never
                # joins is named after the recovery timeout (epoch > 0: a re-formed cluster) or
                # the start-up timeout instead of blocking inside the group's rendezvous
                wait = (rendezvous.recovery_timeout_s() if self.generation > 0
                        else self.timeout_s)
                rendezvous.arrive(self.store, self.generation, self.rank, self.world_size, wait,
                                  f"{self.job_name}:{self.task_index} (rank {self.rank})")
            rendezvous.init_group("gloo", self.rank, self.world_size, self.store,
                                  self.generation, self.timeout_s)
            if self.watcher is not None:
                self.watcher.stop()
            self.watcher = rendezvous.EpochWatcher(self.generation).start()
        wb = self.worker_backend
        if wb is None:
            wb = "gloo"
        # every process of the world must take part in new_group, members or not
        self.worker_group = dist.new_group(self.worker_ranks(), backend=wb)
        self._started = True

    def join(self):
        """ps: serve variables until every worker stopped / shutdown; others: barrier-free no-op."""
        if self.job_name != "ps":
            return None
        from ..parallel.ps_service import ParameterServerService
        svc = ParameterServerService(self.task_index, self.worker_ranks(), device=self.ps_device,
                                     cluster_changed=self.cluster_changed)
        stats = svc.serve()
        return stats

    REJOIN_EXIT_CODE = 75

    @classmethod
    def exit_for_rejoin(cls, stats):
        """A PS task whose cluster moved to a new epoch (a peer died and was restarted) holds
        no state worth keeping -- the chief re-seeds every shard from the latest checkpoint --
        so it leaves as a whole and the launcher starts a fresh one in the new epoch.  Uses
        ``os._exit``: the service thread may still sit in a receive on the broken group."""
        if stats.get("rejoin"):
            print(f"[dtf] cluster moved to a new epoch; parameter server task restarts "
                  f"(exit {cls.REJOIN_EXIT_CODE})", flush=True)
            os._exit(cls.REJOIN_EXIT_CODE)

    def cluster_changed(self):
        """True once the launcher restarted a task (the cluster moved to a new epoch)."""
        return self.watcher is not None and self.watcher.changed

    def restart_group(self, timeout_s=None):
        """Tear down this epoch's process group (a peer died) and join the next epoch; blocks
        until every task -- including the restarted one -- has joined.  Both waits (the
        launcher's epoch bump, the other tasks' arrival) are bounded by ``timeout_s`` (default
        ``DTF_RECOVERY_TIMEOUT_S``): a death nobody restarts raises TimeoutError."""
        if timeout_s is None:
            timeout_s = rendezvous.recovery_timeout_s()
        rendezvous.leave_group()
        rendezvous.wait_for_epoch_after(self.store, self.generation, timeout_s)
        self._started = False
        self.worker_group = None
        self.start()
        return self.generation

    def shutdown(self):
        if self.watcher is not None:
            self.watcher.stop()
        if dist.is_initialized():
            dist.destroy_process_group()
        self._started = False

    @staticmethod
    def create_local_server(config=None, start=True):
        port = int(os.environ.get("MASTER_PORT", "29501"))
        return Server({"worker": [f"127.0.0.1:{port}"]}, "worker", 0, config, start)
