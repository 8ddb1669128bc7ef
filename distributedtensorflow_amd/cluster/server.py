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

Recovery (TF's ``_RecoverableSession`` recreating the session after a PS restart, reference
``run_mnist_distributed.py:146``): the rendezvous TCPStore is created once by the
chief and outlives process groups.  Every (re)join of a rank bumps that rank's join counter in the
store and uses it as the GENERATION of the process group it joins (``PrefixStore("g<n>")``): a
PS task restarted by the launcher after a crash is a new process whose first join is its rank's
second, so it meets the surviving tasks -- which called :meth:`restart_group` when they saw the
failure -- in generation 1 without any extra coordination.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

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
                # the chief hosts the store; every other task (and a restarted one) connects
                self.store = dist.TCPStore(self.host, self.port, None, self.rank == 0,
                                           timeout=datetime.timedelta(seconds=self.timeout_s),
                                           wait_for_workers=False)
            self.generation = int(self.store.add(f"dtf/join/{self.rank}", 1)) - 1
            dist.init_process_group(
                "gloo", store=dist.PrefixStore(f"g{self.generation}", self.store),
                rank=self.rank, world_size=self.world_size,
                timeout=datetime.timedelta(seconds=self.timeout_s))
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
        svc = ParameterServerService(self.task_index, self.worker_ranks(), device=self.ps_device)
        stats = svc.serve()
        return stats

    def restart_group(self):
        """Tear down this generation's process group (a peer died) and join the next one; blocks
        until every task -- including the restarted one -- has joined."""
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:           # the group may already be broken
                pass
        self._started = False
        self.worker_group = None
        self.start()
        return self.generation

    def shutdown(self):
        if dist.is_initialized():
            dist.destroy_process_group()
        self._started = False

    @staticmethod
    def create_local_server(config=None, start=True):
        port = int(os.environ.get("MASTER_PORT", "29501"))
        return Server({"worker": [f"127.0.0.1:{port}"]}, "worker", 0, config, start)
