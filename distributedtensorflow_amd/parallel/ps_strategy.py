"""ParameterServerStrategy (BASELINE.json config 4; reference R6/R13/T6/T7).

Two deployments of the same semantics — variables are OWNED by parameter-server shards, workers
compute gradients, owners apply the optimizer, workers read back the new values:

* **between-graph** (``ParameterServerStrategy(server=Server(...))``): the reference's layout —
  separate ``ps`` tasks run :class:`~.ps_service.ParameterServerService` (``server.join()``);
  workers pull/push over the gloo world (async Hogwild by default, ``sync=True`` =
  SyncReplicasOptimizer aggregation with stale-gradient drop).
* **colocated, synchronous, on RCCL** (no ``server``; one process per GPU under torchrun): the
  PS shards are hosted by the GPU ranks themselves (``num_ps`` owners; 1 = "1 PS + N workers",
  default = every rank owns a byte-balanced slice).  Per step: as soon as a gradient bucket is
  complete during backward, each owner's piece of it is ``reduce``d to its owner over xGMI
  (overlapped with the rest of backward); after backward the owner runs the fused optimizer on
  exactly its slices and ``broadcast``s the updated master slices back.  With num_ps == world
  this is a bucketed reduce-scatter / all-gather step.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .strategy import (BucketedAllReduce, MirroredStrategy, Strategy, _NullReducer,
                       init_process_group_from_env)


class _RemotePSReducer(_NullReducer):
    """Between-graph: push the gradients at step end; the reply carries the updated variables
    (so the NEXT forward pass reads fresh values — TF's read-at-step-start semantics)."""

    applies_update = True

    def __init__(self, space, client):
        super().__init__(space)
        self.client = client

    def apply_remote(self, optimizer):
        params = self.space.order
        return self.client.push([p.grad for p in params], pull=True)


class _ColocatedPSReducer(BucketedAllReduce):
    """Colocated sync PS on RCCL, overlapped with backward.

    The gradient buffer is cut into the same buckets as MirroredStrategy's all-reduce.  When a
    bucket's last gradient lands (post-accumulate hook, during backward) each owner's piece of
    it is ``reduce``d to that owner on RCCL's stream -- the gradient push of the reference's
    ``SyncReplicasOptimizer`` (``templates/00_mnist_replica.py:168-191``) happens while autograd
    is still producing earlier layers.  After backward: each owner applies the fused optimizer
    to the slices it owns and ``broadcast``s the updated master slices (the variable pull)."""

    applies_update = True

    def __init__(self, space, owners_ranges, group=None, bucket_bytes=64 << 20,
                 first_bucket_bytes=4 << 20):
        super().__init__(space, group, bucket_bytes, first_bucket_bytes)
        self.ranges = owners_ranges          # [(owner_rank, start, end)]
        self.rank = dist.get_rank()
        # per bucket: [(owner, start, end)] pieces (bucket ∩ owner range)
        self.pieces = []
        for bs, be, _ in self.buckets:
            self.pieces.append([(o, max(bs, s), min(be, e)) for o, s, e in owners_ranges
                                if min(be, e) > max(bs, s)])

    def _launch(self, b):
        if self.launched[b]:
            return
        self.launched[b] = True
        for o, s, e in self.pieces[b]:
            self.works.append((dist.reduce(self.space.grad[s:e], dst=o, group=self.group,
                                           async_op=True), None, None))

    def grad_scale(self):
        return 1.0 / self.world

    def apply_remote(self, optimizer):
        for o, s, e in self.ranges:
            if o == self.rank and e > s:
                optimizer._apply(self.grad_scale(), (s, e))
        works = [dist.broadcast(self.space.master[s:e], src=o, group=self.group, async_op=True)
                 for o, s, e in self.ranges if e > s]
        for w in works:
            w.wait()
        self.space.refresh_shadow()
        return None


def balanced_ranges(space, num_owners, owner_ranks):
    """Contiguous, variable-aligned slices of the flat buffer with ~equal element counts."""
    total = space.numel
    bounds, target, k = [0], total / num_owners, 1
    for o in space.offsets[1:]:
        if k < num_owners and o >= target * k:
            bounds.append(o)
            k += 1
    while len(bounds) < num_owners:
        bounds.append(total)
    bounds.append(total)
    return [(owner_ranks[i], bounds[i], bounds[i + 1]) for i in range(num_owners)]


class ParameterServerStrategy(Strategy):
    def __init__(self, cluster_resolver=None, server=None, num_ps=None, sync=None,
                 replicas_to_aggregate=None, variable_placement="balanced", device=None,
                 data_plane=None, bucket_mb=64, first_bucket_mb=4):
        self.server = server
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.first_bucket_bytes = int(first_bucket_mb * (1 << 20))
        self.data_plane = data_plane
        self.variable_placement = variable_placement
        self.replicas_to_aggregate = replicas_to_aggregate
        self._client = None
        if server is not None:
            # between-graph: this process is a worker of a PS cluster
            local = int(os.environ.get("LOCAL_RANK", "0"))
            if device is None:
                device = (torch.device("cuda", local % max(torch.cuda.device_count(), 1))
                          if torch.cuda.is_available() else torch.device("cpu"))
            if device.type == "cuda":
                torch.cuda.set_device(device)
            super().__init__(device)
            self.sync = bool(sync)
            self.mode = "between_graph"
        else:
            local = int(os.environ.get("LOCAL_RANK", "0"))
            if torch.cuda.is_available():
                torch.cuda.set_device(local)
                device = torch.device("cuda", local)
            else:
                device = torch.device("cpu")
            super().__init__(device)
            if int(os.environ.get("WORLD_SIZE", "1")) > 1:
                init_process_group_from_env()
            self.sync = True if sync is None else bool(sync)
            if not self.sync:
                raise ValueError("colocated ParameterServerStrategy is synchronous; use a "
                                 "between-graph cluster (Server with ps tasks) for async PS")
            self.mode = "colocated"
            w = dist.get_world_size() if dist.is_initialized() else 1
            self.num_ps = min(num_ps or w, w)

    # -- topology
    @property
    def num_replicas_in_sync(self):
        if self.mode == "between_graph":
            return len(self.server.worker_ranks()) if self.sync else 1
        return dist.get_world_size() if dist.is_initialized() else 1

    @property
    def replica_id(self):
        if self.mode == "between_graph":
            return self.server.worker_ranks().index(self.server.rank)
        return dist.get_rank() if dist.is_initialized() else 0

    @property
    def is_chief(self):
        return self.server.is_chief if self.mode == "between_graph" else self.replica_id == 0

    # -- hooks used by Optimizer.build
    def make_gradient_reducer(self, space):
        if self.mode == "between_graph":
            from .ps_service import PSClient
            self._client = PSClient(self.server.ps_ranks(), policy=self.variable_placement,
                                    space=space, data_plane=self.data_plane)
            return _RemotePSReducer(space, self._client)
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return _NullReducer(space)
        ranges = balanced_ranges(space, self.num_ps, list(range(self.num_ps)))
        return _ColocatedPSReducer(space, ranges, None, self.bucket_bytes,
                                   self.first_bucket_bytes)

    def broadcast_space(self, space):
        if self.mode == "colocated":
            if dist.is_initialized() and dist.get_world_size() > 1:
                dist.broadcast(space.master, 0)
                space.refresh_shadow()

    def register_with_ps(self, optimizer, global_step=0, restored_slots=False):
        """Chief: ship variables + optimizer config (+ the optimizer slots just restored from a
        checkpoint) to the PS shards; others: wait for it."""
        if self.mode != "between_graph":
            return
        params = optimizer.space.order
        if self.is_chief:
            slots = None
            if restored_slots and optimizer.slots:
                slots = {s.name: [optimizer.space.view_of(s.buf, p) for p in params]
                         for s in optimizer.slots}
            self._client.register(params, optimizer.get_config(), sync=self.sync,
                                  replicas_to_aggregate=self.replicas_to_aggregate,
                                  global_step=int(global_step), slots=slots,
                                  iterations=optimizer.iterations if restored_slots else None)
        self._client.wait_ready(params)
        self._client.pull()          # every worker starts from the PS values

    def recover_cluster(self, optimizer):
        """A task of the cluster died (a PS crashed and is being restarted by the launcher):
        leave the broken process group, join the next generation (blocks until the restarted
        PS joins too) and re-map the new shard's buffers.  The caller restores the checkpoint
        and calls :meth:`register_with_ps` again (chief re-initialises the PS; others wait)."""
        if self.mode != "between_graph":
            raise RuntimeError("cluster recovery is for between-graph parameter servers")
        self.server.restart_group()
        from .ps_service import PSClient
        old = self._client
        self._client = PSClient(self.server.ps_ranks(), policy=self.variable_placement,
                                space=old.space, data_plane=self.data_plane)
        reducer = getattr(optimizer, "_reducer", None)
        if reducer is not None and hasattr(reducer, "client"):
            reducer.client = self._client
        return self.server.generation

    @property
    def ps_client(self):
        return self._client

    def barrier(self):
        if self.mode == "colocated" and dist.is_initialized():
            dist.barrier()


# tf.compat.v1 naming
ParameterServerStrategyV1 = ParameterServerStrategy
CentralStorageStrategy = MirroredStrategy
