"""Cluster description: ``config.json`` / comma-separated flags / ``TF_CONFIG``.

Reference: ``Config`` in ``run_mnist_distributed.py:14-43`` (JSON ``{"ps": {...}, "workers":
{...}}``; task order = JSON insertion order, not the ``worker:N`` suffix), comma-list flags in
``templates/00_mnist_replica.py:80-83,104-111``, and ``tf.train.ClusterSpec``.
``TF_CONFIG`` (``{"cluster": {...}, "task": {"type", "index"}}``) is the tf.distribute form.

Process layout used by this framework (one OS process per task, one GPU per process):
global rank = position in the job order ``chief, worker, ps, evaluator`` — so the chief worker
is rank 0 and hosts the rendezvous store; every task joins one torch.distributed world.
"""
from __future__ import annotations

import json
import os
from collections import OrderedDict

JOB_ORDER = ("chief", "worker", "ps", "evaluator")


class Config:
    """Reference-compatible loader of ``config.json`` (``run_mnist_distributed.py:14-43``)."""

    def __init__(self, file_path="config.json"):
        self.file_path = file_path
        with open(file_path) as f:
            self.json = json.load(f, object_pairs_hook=OrderedDict)
        missing = [k for k in ("ps", "workers") if k not in self.json]
        if missing:
            raise AttributeError(
                'Please provide a value for "{0}" configuration key in the config.json file!'
                .format(missing[0]))
        self.ps = self.json["ps"]
        self.workers = self.json["workers"]

    def get_workers_with_addresses(self):
        return tuple(self.workers.keys()), tuple(self.workers.values())

    def get_ps_with_addresses(self):
        return tuple(self.ps.keys()), tuple(self.ps.values())

    def get_ps_and_worker_hosts(self):
        return self.get_ps_with_addresses()[1], self.get_workers_with_addresses()[1]

    def cluster_spec(self) -> "ClusterSpec":
        ps, workers = self.get_ps_and_worker_hosts()
        return ClusterSpec({"ps": list(ps), "worker": list(workers)})


class ClusterSpec:
    """``tf.train.ClusterSpec``: job name -> ordered task addresses."""

    def __init__(self, cluster):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.as_dict()
        self._jobs: "OrderedDict[str, list]" = OrderedDict()
        for job, tasks in cluster.items():
            if isinstance(tasks, dict):
                tasks = [tasks[k] for k in sorted(tasks, key=int)]
            self._jobs[job] = list(tasks)

    @property
    def jobs(self):
        return [j for j in JOB_ORDER if j in self._jobs] + \
               [j for j in self._jobs if j not in JOB_ORDER]

    def job_tasks(self, job):
        return list(self._jobs.get(job, []))

    def num_tasks(self, job):
        return len(self._jobs.get(job, []))

    def task_address(self, job, index):
        return self._jobs[job][index]

    def as_dict(self):
        return {j: list(t) for j, t in self._jobs.items()}

    def __eq__(self, other):
        return isinstance(other, ClusterSpec) and self.as_dict() == other.as_dict()

    def __repr__(self):
        return f"ClusterSpec({self.as_dict()})"

    # -- global rank layout
    def world_size(self) -> int:
        return sum(len(t) for t in self._jobs.values())

    def rank_of(self, job, index) -> int:
        r = 0
        for j in self.jobs:
            if j == job:
                if not 0 <= index < len(self._jobs[j]):
                    raise ValueError(f"task index {index} out of range for job {job!r}")
                return r + index
            r += len(self._jobs[j])
        raise ValueError(f"unknown job {job!r}")

    def task_of(self, rank):
        r = rank
        for j in self.jobs:
            n = len(self._jobs[j])
            if r < n:
                return j, r
            r -= n
        raise ValueError(f"rank {rank} out of range")

    def chief(self):
        """(job, index) of the chief: ``chief:0`` if present else ``worker:0`` (reference rule
        ``is_chief = task_index == 0``, ``run_mnist_distributed.py:106``)."""
        return ("chief", 0) if self.num_tasks("chief") else ("worker", 0)

    def hosts(self):
        """The distinct hosts of the cluster's tasks (loopback names folded together)."""
        out = set()
        for job in self.jobs:
            for addr in self.job_tasks(job):
                h = split_host_port(addr)[0].lower()
                out.add("localhost" if h in ("localhost", "127.0.0.1", "::1", "0.0.0.0") else h)
        return out

    def single_host(self):
        """True when every task runs on one host: the parameter servers' device data plane
        (hipIpc / shared memory) is only valid there; other clusters use gloo over TCP."""
        return len(self.hosts()) <= 1

    def rendezvous_address(self):
        job, idx = self.chief()
        host, port = split_host_port(self.task_address(job, idx))
        return host, port


def split_host_port(addr: str):
    addr = addr.replace("grpc://", "").replace("dtf://", "")
    host, _, port = addr.rpartition(":")
    if not host:
        raise ValueError(f"address {addr!r} is not host:port")
    return host, int(port)


def from_flags(ps_hosts: str, worker_hosts: str, chief_hosts: str = "") -> ClusterSpec:
    d = OrderedDict()
    if chief_hosts:
        d["chief"] = [h for h in chief_hosts.split(",") if h]
    d["worker"] = [h for h in worker_hosts.split(",") if h]
    if ps_hosts:
        d["ps"] = [h for h in ps_hosts.split(",") if h]
    return ClusterSpec(d)


def from_tf_config(tf_config=None):
    """Returns (ClusterSpec, job, index) from TF_CONFIG (string, dict or env)."""
    if tf_config is None:
        tf_config = os.environ.get("TF_CONFIG")
    if not tf_config:
        raise ValueError("TF_CONFIG is not set")
    cfg = json.loads(tf_config) if isinstance(tf_config, str) else tf_config
    spec = ClusterSpec(cfg.get("cluster", {}))
    task = cfg.get("task", {})
    return spec, task.get("type", "worker"), int(task.get("index", 0))
