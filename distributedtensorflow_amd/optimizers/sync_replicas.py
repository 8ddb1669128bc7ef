"""``tf.train.SyncReplicasOptimizer`` (``templates/00_mnist_replica.py:168-191``).

Wraps an optimizer; under a between-graph :class:`ParameterServerStrategy` it switches the PS
shards to synchronous aggregation: per global step the PS averages the first
``replicas_to_aggregate`` gradients computed at that step (``total_num_replicas`` may be larger:
backup workers), drops stale ones, applies once and releases the workers (the token queue).
Under Mirrored/MultiWorkerMirrored (and the colocated PS) training is already synchronous over
every replica, so it delegates -- and raises if asked for backup workers
(``replicas_to_aggregate < replicas``), which only the arrival-order between-graph PS provides.  The queue-runner / init-token API of TF1 is provided as no-ops for drop-in use.
"""
from __future__ import annotations


class _NoOp:
    def __call__(self, *a, **k):
        return None

    def run(self, *a, **k):
        return None


class SyncReplicasOptimizer:
    def __init__(self, opt, replicas_to_aggregate, total_num_replicas=None, variable_averages=None,
                 variables_to_average=None, use_locking=False, name="sync_replicas"):
        from ..parallel.strategy import get_strategy
        self._opt = opt
        self.replicas_to_aggregate = int(replicas_to_aggregate)
        self.total_num_replicas = int(total_num_replicas or replicas_to_aggregate)
        if self.replicas_to_aggregate > self.total_num_replicas:
            raise ValueError("replicas_to_aggregate > total_num_replicas")
        self.name = name
        strat = get_strategy()
        if getattr(strat, "mode", None) == "between_graph":
            strat.sync = True
            strat.replicas_to_aggregate = self.replicas_to_aggregate
        elif strat.num_replicas_in_sync > 1 and \
                self.replicas_to_aggregate < strat.num_replicas_in_sync:
            # collective strategies (RCCL all-reduce / reduce-to-owner) need EVERY replica's
            # gradient each step: "first N of M" backup-worker aggregation only exists on the
            # between-graph PS, whose owners take gradients in arrival order
            raise ValueError(
                f"replicas_to_aggregate={self.replicas_to_aggregate} < "
                f"{strat.num_replicas_in_sync} replicas: backup workers need the between-graph "
                f"ParameterServerStrategy (Server with ps tasks); {type(strat).__name__} "
                f"aggregates every replica each step")
        self.local_step_init_op = _NoOp()
        self.chief_init_op = _NoOp()
        self.ready_for_local_init_op = _NoOp()

    def __getattr__(self, name):
        return getattr(self._opt, name)

    def minimize(self, loss, global_step=None, var_list=None):
        return self._opt.minimize(loss, global_step=global_step, var_list=var_list)

    def compute_gradients(self, loss, var_list=None):
        return self._opt.compute_gradients(loss, var_list)

    def apply_gradients(self, grads_and_vars=None, global_step=None):
        return self._opt.apply_gradients(grads_and_vars, global_step)

    def get_chief_queue_runner(self):
        return _NoOp()

    def get_init_tokens_op(self, num_tokens=-1):
        return _NoOp()

    def make_session_run_hook(self, is_chief, num_tokens=-1):
        from ..train.hooks import SessionRunHook
        return SessionRunHook()
