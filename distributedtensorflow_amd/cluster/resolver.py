"""Cluster resolvers: turn a cluster description into a torch.distributed world.

``TFConfigClusterResolver`` / ``SimpleClusterResolver`` mirror tf.distribute's; ``export_torch_env``
writes ``MASTER_ADDR/MASTER_PORT/WORLD_SIZE/RANK/LOCAL_RANK`` so every strategy uses the same
TCPStore rendezvous (hosted by the chief, rank 0).  ``LOCAL_RANK`` = index of this task among the
tasks that share its host (one process per GPU).
"""
from __future__ import annotations

import os

from .spec import ClusterSpec, from_tf_config, split_host_port


class SimpleClusterResolver:
    def __init__(self, cluster_spec: ClusterSpec, task_type="worker", task_id=0,
                 rpc_layer="dtf"):
        self._spec = ClusterSpec(cluster_spec)
        self.task_type = task_type
        self.task_id = int(task_id)
        self.rpc_layer = rpc_layer

    def cluster_spec(self) -> ClusterSpec:
        return self._spec

    @property
    def rank(self):
        return self._spec.rank_of(self.task_type, self.task_id)

    @property
    def world_size(self):
        return self._spec.world_size()

    def local_rank(self):
        me = self._spec.task_address(self.task_type, self.task_id)
        host = split_host_port(me)[0]
        idx = 0
        for r in range(self.rank):
            j, i = self._spec.task_of(r)
            if split_host_port(self._spec.task_address(j, i))[0] == host:
                idx += 1
        return idx

    def master(self):
        host, port = self._spec.rendezvous_address()
        return f"{self.rpc_layer}://{host}:{port}"


class TFConfigClusterResolver(SimpleClusterResolver):
    def __init__(self, tf_config=None):
        spec, job, idx = from_tf_config(tf_config)
        super().__init__(spec, job, idx)


def export_torch_env(resolver=None, force=False):
    if resolver is None:
        resolver = TFConfigClusterResolver()
    host, port = resolver.cluster_spec().rendezvous_address()
    env = {"MASTER_ADDR": host, "MASTER_PORT": str(port), "WORLD_SIZE": str(resolver.world_size),
           "RANK": str(resolver.rank), "LOCAL_RANK": str(resolver.local_rank())}
    for k, v in env.items():
        if force or k not in os.environ:
            os.environ[k] = v
    return env
