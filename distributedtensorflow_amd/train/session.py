"""``MonitoredTrainingSession`` / ``Supervisor`` for eager step functions.

Reference: ``run_mnist_distributed.py:118-161`` (MTS + StopAtStepHook, chief logs every step),
``templates/00_mnist_replica.py:193-240`` (Supervisor, prepare_or_wait_for_session),
``templates/00_between…:40-52`` (MTS with checkpoint_dir).  SURVEY R14/R16/R17, T12.

A "train op" is a Python callable performing one training step (forward, backward, optimizer
update through the active strategy).  ``run(fetches)`` accepts a callable, a list/tuple/dict of
callables, :class:`~.global_step.GlobalStep` objects (resolved after the step), or strings naming
keys of the dict returned by the first callable — so the reference's
``mon_sess.run([train_op, loss, global_step])`` becomes ``run([train_op, "loss", global_step])``.

Session creation follows TF1: the chief restores the latest checkpoint in ``checkpoint_dir`` (or
initialises) and, under a between-graph ParameterServerStrategy, ships the variables to the PS;
non-chief workers wait for the chief (``recovery_wait_secs`` polling is implicit in the PS
rendezvous).  Recoverable failures during ``run`` (a dropped RCCL/gloo peer, an injected fault)
re-create the session from the latest checkpoint up to ``max_recovery_attempts`` times.
"""
from __future__ import annotations

import os
import time

import torch

from . import global_step as gs_mod
from .checkpoint import Saver, latest_checkpoint
from .hooks import (CheckpointSaverHook, InjectedFault, SessionRunContext, SessionRunValues,
                    StepCounterHook, SummarySaverHook)


class GPUOptions:
    """``tf.GPUOptions`` subset.  ``per_process_gpu_memory_fraction`` caps this process's share
    of the device's HBM in PyTorch's caching allocator; ``allow_growth`` is the allocator's native
    behaviour (memory is reserved on demand, never up front); ``visible_device_list`` picks the
    device by index into the listed ids (the process keeps one GPU, as everywhere here)."""

    def __init__(self, per_process_gpu_memory_fraction=0.0, allow_growth=True,
                 visible_device_list=""):
        self.per_process_gpu_memory_fraction = float(per_process_gpu_memory_fraction or 0.0)
        self.allow_growth = bool(allow_growth)
        self.visible_device_list = str(visible_device_list or "")

    def apply(self, placed_on=None):
        """``placed_on``: the device the session's variables already live on.  Switching the
        current device away from it would send the native kernels to one device's stream with
        the other device's pointers, so a ``visible_device_list`` naming a different device is
        refused instead of applied."""
        if not torch.cuda.is_available():
            return None
        dev = torch.cuda.current_device()
        if self.visible_device_list:
            ids = [int(t) for t in self.visible_device_list.split(",") if t.strip()]
            dev = ids[0]
            if placed_on is not None and placed_on.type == "cuda" and \
                    (placed_on.index if placed_on.index is not None else 0) != dev:
                raise ValueError(f"GPUOptions(visible_device_list={self.visible_device_list!r}) "
                                 f"selects cuda:{dev}, but the variables were already created "
                                 f"on {placed_on}; pick the device before building the model "
                                 f"(or set HIP_VISIBLE_DEVICES)")
            torch.cuda.set_device(dev)
        if 0.0 < self.per_process_gpu_memory_fraction <= 1.0:
            torch.cuda.set_per_process_memory_fraction(self.per_process_gpu_memory_fraction, dev)
        return dev


def parse_device_filter(spec):
    """'/job:ps', '/job:worker/task:3', '/job:worker/replica:0/task:1' -> (job, task or None).
    Fields TF allows but this framework has one of (replica, device) are accepted and ignored."""
    job, task = None, None
    for part in str(spec).strip().strip("/").split("/"):
        if not part:
            continue
        key, _, val = part.partition(":")
        key = key.lower()
        if key == "job":
            job = val
        elif key == "task":
            task = int(val)
        elif key in ("replica", "device", "cpu", "gpu"):
            pass
        else:
            raise ValueError(f"bad device filter {spec!r}: unknown field {key!r}")
    if job is None:
        raise ValueError(f"bad device filter {spec!r}: no /job:")
    return job, task


class ConfigProto:
    """``tf.ConfigProto`` subset (``run_mnist_distributed.py:122-124``,
    ``templates/00_mnist_replica.py:213-217``).  Thread counts are applied to torch's CPU pools;
    ``gpu_options`` (a :class:`GPUOptions` or a dict of its fields) to the device allocator.

    ``device_filters`` (e.g. ``["/job:ps", "/job:worker/task:1"]``): the tasks this session may
    depend on.  :meth:`device_visible` answers for a (job, task); the between-graph PS client only
    ever talks to PS tasks and its own task, so the reference's usual filter is always satisfied,
    and a filter that hides every PS task while variables live there is refused at session start
    (TF would hang waiting for an invisible device).  ``log_device_placement`` prints where each
    variable lives when the session is created."""

    def __init__(self, allow_soft_placement=True, log_device_placement=False,
                 intra_op_parallelism_threads=0, inter_op_parallelism_threads=0,
                 device_filters=None, gpu_options=None, **kw):
        self.allow_soft_placement = allow_soft_placement
        self.log_device_placement = log_device_placement
        self.intra_op_parallelism_threads = intra_op_parallelism_threads
        self.inter_op_parallelism_threads = inter_op_parallelism_threads
        self.device_filters = list(device_filters or [])
        self._filters = [parse_device_filter(f) for f in self.device_filters]
        if isinstance(gpu_options, dict):
            gpu_options = GPUOptions(**gpu_options)
        self.gpu_options = gpu_options
        self.extra = kw

    def device_visible(self, job, task=None):
        if not self._filters:
            return True
        return any(j == job and (t is None or task is None or t == task) for j, t in self._filters)

    def check_placement(self, strategy):
        """Refuse filters that hide the parameter servers this session's variables live on."""
        server = getattr(strategy, "server", None)
        if server is None or not self._filters:
            return
        num_ps = server.cluster.num_tasks("ps")
        if num_ps <= 0:
            return
        if not any(self.device_visible("ps", t) for t in range(num_ps)):
            raise ValueError(f"device_filters {self.device_filters} hide every /job:ps task, but "
                             f"the variables live on {num_ps} parameter server(s)")

    def apply(self, placed_on=None):
        # clamp to the CPUs this process may use (utils.cpu.usable_cpus): the reference passes
        # os.cpu_count(), which on a shared many-core GPU host is far above the CPU quota
        from ..utils.cpu import usable_cpus
        cap = usable_cpus()
        if self.intra_op_parallelism_threads:
            torch.set_num_threads(min(int(self.intra_op_parallelism_threads), cap))
        if self.inter_op_parallelism_threads:
            try:
                torch.set_num_interop_threads(min(int(self.inter_op_parallelism_threads), cap))
            except RuntimeError:
                pass   # can only be set once per process
        if self.gpu_options is not None:
            self.gpu_options.apply(placed_on)


def log_placement(model=None, optimizer=None, strategy=None, out=None):
    """``log_device_placement``: one line per variable -- its name, shape and where it lives
    (the owning PS task for sharded variables, else this replica's device)."""
    import sys
    out = out or sys.stderr
    params = []
    if optimizer is not None and getattr(optimizer, "space", None) is not None:
        params = list(optimizer.space.order)
    elif model is not None:
        params = list(model.parameters())
    owner = getattr(strategy, "variable_owner", None)
    for p in params:
        name = getattr(p, "_dtf_name", None) or getattr(p, "name", None) or "variable"
        where = owner(p) if callable(owner) else None
        where = where or str(p.device)
        print(f"{name} {tuple(p.shape)}: {where}", file=out)


RunConfig = ConfigProto


class Scaffold:
    def __init__(self, model=None, optimizer=None, global_step=None, saver=None, init_fn=None):
        self.model, self.optimizer, self.global_step = model, optimizer, global_step
        self.saver, self.init_fn = saver, init_fn

    def finalize(self):
        if self.global_step is None:
            self.global_step = gs_mod.get_or_create_global_step()
        if self.saver is None and (self.model is not None or self.optimizer is not None):
            self.saver = Saver(model=self.model, optimizer=self.optimizer,
                               global_step=self.global_step)
        return self


class _Session:
    """The object hooks see (``run_context.session``)."""

    def __init__(self, scaffold, strategy, is_chief, checkpoint_dir, summary_writer):
        self.scaffold = scaffold
        self.strategy = strategy
        self.is_chief = is_chief
        self.checkpoint_dir = checkpoint_dir
        self.summary_writer = summary_writer
        self.last_results = None

    @property
    def global_step(self):
        return self.scaffold.global_step

    @property
    def saver(self):
        return self.scaffold.saver

    def save_checkpoint(self, path, step, saver=None):
        saver = saver or self.saver
        opt = self.scaffold.optimizer
        if opt is not None and opt.space is not None:
            opt.synchronize_variables()
            if getattr(self.strategy, "collective", False):
                # collective: every rank is here (step-triggered saver hook on every rank); a
                # sharded parameter server completes its slot shards on every rank first
                opt.gather_state()
                if not self.is_chief:
                    return None
        values = None
        client = getattr(self.strategy, "ps_client", None)
        if client is not None and client.params is not None:
            gstep, values, slots = client.get_state()
            for sname, per in slots.items():
                for vname, t in per.items():
                    values[f"{vname}/{sname}"] = t
            self.global_step.assign(gstep)
        return saver.save(None, path, global_step=step, values=values)

    def run(self, fetches, feed_dict=None):
        return _execute(fetches, feed_dict, self)


def _execute(fetches, feed_dict, session):
    first_result = {}

    def ev(f):
        nonlocal first_result
        if isinstance(f, gs_mod.GlobalStep):
            return None   # resolved after all callables ran
        if callable(f):
            r = f(**feed_dict) if feed_dict else f()
            if isinstance(r, dict) and not first_result:
                first_result = r
            return r
        return f

    def resolve(f, v):
        if isinstance(f, gs_mod.GlobalStep):
            return f.value()
        if isinstance(f, str):
            r = first_result.get(f)
            return float(r.detach()) if isinstance(r, torch.Tensor) and r.numel() == 1 else r
        return v

    if isinstance(fetches, (list, tuple)):
        vals = [ev(f) if not isinstance(f, str) else None for f in fetches]
        out = [resolve(f, v) for f, v in zip(fetches, vals)]
        out = type(fetches)(out) if isinstance(fetches, tuple) else out
    elif isinstance(fetches, dict):
        vals = {k: (ev(f) if not isinstance(f, str) else None) for k, f in fetches.items()}
        out = {k: resolve(f, vals[k]) for k, f in fetches.items()}
    else:
        out = resolve(fetches, ev(fetches))
    if session is not None:
        session.last_named = first_result   # what hooks (summaries, NaN check, logging) see
    return out


def _recoverable(exc):
    """Errors TF's _RecoverableSession would recreate the session for -- matched by TYPE, never
    by message text: injected faults (in-process checkpoint rollback), and communication
    failures (a peer died: this package's CommError / ClusterChanged, both ConnectionErrors,
    torch.distributed's DistError family, a data-plane TimeoutError).  Communication failures
    are recoverable only when a launcher restarts failed tasks (``DTF_MAX_RESTARTS`` with the
    launcher-hosted store): without one, waiting for the cluster to re-form would only hang."""
    import torch.distributed as dist

    from ..cluster import rendezvous
    if isinstance(exc, InjectedFault):
        return True
    if isinstance(exc, (ConnectionError, TimeoutError, getattr(dist, "DistError", ()))):
        return rendezvous.recovery_enabled()
    return False


def _maybe_hard_fault(strategy, step):
    """``DTF_FAULT_SIGKILL=<job>:<index>@<step>`` (tests, SURVEY §5.3 fault injection): this task
    dies by SIGKILL -- no cleanup, like a preempted host -- when the global step reaches
    ``step``, in its first incarnation only (``DTF_RESTART_COUNT`` = 0).  ``job`` is ``worker`` /
    ``ps`` for between-graph clusters, ``rank`` for collective worlds."""
    spec = os.environ.get("DTF_FAULT_SIGKILL", "")
    if not spec or int(os.environ.get("DTF_RESTART_COUNT", "0") or 0):
        return
    who, _, at = spec.partition("@")
    job, _, idx = who.partition(":")
    server = getattr(strategy, "server", None)
    if server is not None:
        me = (server.job_name, server.task_index)
    else:
        me = ("rank", int(os.environ.get("RANK", "0")))
    if me == (job, int(idx)) and step >= int(at):
        import signal
        print(f"[dtf] fault injection: SIGKILL {job}:{idx} at global step {step}", flush=True)
        os.kill(os.getpid(), signal.SIGKILL)


def _comm_check():
    from ..parallel import watchdog
    watchdog.check()


class MonitoredTrainingSession:
    # the exception types _recoverable() accepts (communication ones only under a launcher
    # that restarts failed tasks)
    RECOVERABLE = (InjectedFault, ConnectionError, TimeoutError)

    def __init__(self, master="", is_chief=True, checkpoint_dir=None, scaffold=None, hooks=None,
                 chief_only_hooks=None, save_checkpoint_secs=600, save_summaries_steps=100,
                 save_summaries_secs=None, config=None, stop_grace_period_secs=120,
                 log_step_count_steps=100, max_wait_secs=7200, save_checkpoint_steps=None,
                 summary_dir=None, model=None, optimizer=None, global_step=None, strategy=None,
                 max_recovery_attempts=3):
        from ..parallel.strategy import get_strategy
        self.master = master
        self.is_chief = is_chief
        self.checkpoint_dir = checkpoint_dir
        self.scaffold = (scaffold or Scaffold(model, optimizer, global_step)).finalize()
        self.strategy = strategy or get_strategy()
        self.config = config
        self.max_recovery_attempts = max_recovery_attempts
        self.hooks = list(hooks or [])
        self._writer = None
        collective = bool(getattr(self.strategy, "collective", False))
        if checkpoint_dir and (save_checkpoint_secs or save_checkpoint_steps) and \
                (is_chief or collective):
            if collective and not save_checkpoint_steps:
                # every replica must enter the (collective) save at the same step: a wall-clock
                # trigger would fire at different steps on different ranks
                save_checkpoint_steps = max(1, int(os.environ.get("DTF_COLLECTIVE_SAVE_STEPS",
                                                                  "1000")))
            self.hooks.append(CheckpointSaverHook(checkpoint_dir, save_checkpoint_secs
                                                  if not save_checkpoint_steps else None,
                                                  save_checkpoint_steps))
        if is_chief:
            self.hooks += list(chief_only_hooks or [])
            sdir = summary_dir or checkpoint_dir
            if sdir:
                from ..summary.events import EventFileWriter
                self._writer = EventFileWriter(sdir)
            if sdir and log_step_count_steps:
                self.hooks.append(StepCounterHook(every_n_steps=log_step_count_steps))
            if sdir and (save_summaries_steps or save_summaries_secs):
                self.hooks.append(SummarySaverHook(save_summaries_steps, save_summaries_secs))
        self._session = None
        self._should_stop = False
        self._closed = False
        self.recoveries = 0
        self._create()

    # -- creation / recovery
    def _placed_on(self):
        opt = self.scaffold.optimizer
        if opt is not None and getattr(opt, "space", None) is not None:
            return opt.space.device
        if self.scaffold.model is not None:
            p = next(iter(self.scaffold.model.parameters()), None)
            return p.device if p is not None else None
        return None

    def _create(self):
        if self.config is not None and hasattr(self.config, "apply"):
            self.config.apply(self._placed_on())
        sc = self.scaffold
        if self.config is not None and hasattr(self.config, "check_placement"):
            self.config.check_placement(self.strategy)
        restored = False
        if self.is_chief and self.checkpoint_dir and sc.saver is not None:
            ckpt = latest_checkpoint(self.checkpoint_dir)
            if ckpt:
                sc.saver.restore(None, ckpt, strict=False)
                restored = True
        if sc.init_fn is not None and not restored:
            sc.init_fn(self)
        if getattr(self.strategy, "collective", False) and sc.optimizer is not None:
            # synchronous replicas: everyone continues from the chief's (restored) state
            self.strategy.sync_after_restore(sc.optimizer, sc.global_step, restored=restored)
        if sc.optimizer is not None and hasattr(self.strategy, "register_with_ps"):
            self.strategy.register_with_ps(sc.optimizer, sc.global_step.value())
            client = getattr(self.strategy, "ps_client", None)
            if client is not None:
                sc.global_step.assign(client.global_step)
        if self.config is not None and getattr(self.config, "log_device_placement", False):
            log_placement(sc.model, sc.optimizer, self.strategy)
        self._session = _Session(sc, self.strategy, self.is_chief, self.checkpoint_dir,
                                 self._writer)
        for h in self.hooks:
            h.begin()
        for h in self.hooks:
            h.after_create_session(self._session, None)

    def _rejoin(self, state):
        """The cluster re-formation step of a recovery, done at most once per recovery: a retry
        after a later phase failed (restore, PS registration, the post-restore sync) does not
        leave the epoch it already joined -- ``restart_group`` would wait for an epoch after it,
        which only comes if the launcher restarts another task -- unless the cluster moved on
        again meanwhile (``cluster_changed``)."""
        strat = self.strategy
        changed = getattr(strat, "cluster_changed", None)
        if "epoch" not in state or (changed is not None and changed()):
            state["epoch"] = strat.recover_cluster(self.scaffold.optimizer)
        return state["epoch"]

    def _recover(self, exc=None, state=None):
        if state is None:
            state = {}
        if not state.get("counted"):
            self.recoveries += 1          # one recovery, however many retries it takes
            state["counted"] = True
        strat = self.strategy
        sc = self.scaffold
        if exc is not None and not isinstance(exc, InjectedFault) and \
                getattr(strat, "collective", False) and hasattr(strat, "recover_cluster"):
            # a replica of the synchronous world died and was restarted: re-form the world in
            # the new epoch, rebuild the reducer, the chief restores the latest checkpoint and
            # every replica continues from the chief's state (the restarted one does the same
            # from its MonitoredTrainingSession creation)
            print(f"[dtf] recovering from {type(exc).__name__}: {exc}", flush=True)
            epoch = self._rejoin(state)
            ckpt = latest_checkpoint(self.checkpoint_dir) if self.checkpoint_dir else None
            restored = False
            if self.is_chief and ckpt and sc.saver is not None:
                sc.saver.restore(None, ckpt, strict=False)
                restored = True
            strat.sync_after_restore(sc.optimizer, sc.global_step, restored=restored)
            # the restarted replica runs after_create_session (its initial checkpoint save is a
            # collective under a sharded PS): the survivors mirror it
            for h in self.hooks:
                h.after_create_session(self._session, None)
            print(f"[dtf] recovered: generation {epoch}, restored="
                  f"{ckpt if self.is_chief else 'from chief'}, global step "
                  f"{sc.global_step.value()}", flush=True)
            return
        if exc is not None and not isinstance(exc, InjectedFault) and \
                getattr(strat, "mode", None) == "between_graph" and \
                hasattr(strat, "recover_cluster") and sc.optimizer is not None:
            # a task died: next process-group generation (the launcher restarts a crashed PS),
            # chief restores the latest checkpoint and re-initialises the PS shards with it,
            # the other workers wait for that and pull
            print(f"[dtf] recovering from {type(exc).__name__}: {exc}", flush=True)
            gen = self._rejoin(state)
            restored = False
            ckpt = latest_checkpoint(self.checkpoint_dir) if self.checkpoint_dir else None
            if self.is_chief and ckpt and sc.saver is not None:
                sc.saver.restore(None, ckpt, strict=False)
                restored = True
            from ..cluster import rendezvous
            strat.register_with_ps(sc.optimizer, sc.global_step.value(), restored_slots=restored,
                                   timeout_s=rendezvous.recovery_timeout_s())
            client = getattr(strat, "ps_client", None)
            if client is not None:
                sc.global_step.assign(client.global_step)
                self._session.strategy = strat
            print(f"[dtf] recovered: generation {gen}, restored={ckpt if restored else None}, "
                  f"global step {sc.global_step.value()}", flush=True)
            return
        ckpt = latest_checkpoint(self.checkpoint_dir) if self.checkpoint_dir else None
        if ckpt and self.scaffold.saver is not None:
            self.scaffold.saver.restore(None, ckpt, strict=False)
            client = getattr(self.strategy, "ps_client", None)
            if client is not None and self.is_chief:
                client.set_state(self.scaffold.global_step.value())

    # -- public API
    @property
    def global_step(self):
        return self.scaffold.global_step

    def should_stop(self):
        return self._should_stop or self._closed

    def run(self, fetches, feed_dict=None, options=None, run_metadata=None):
        attempts = 0
        while True:
            ctx = SessionRunContext(fetches, self._session)
            for h in self.hooks:
                h.before_run(ctx)
            if ctx.stop_requested:
                self._should_stop = True
                return None
            try:
                changed = getattr(self.strategy, "cluster_changed", None)
                if changed is not None and changed():
                    from ..cluster.rendezvous import ClusterChanged
                    raise ClusterChanged("a task of the cluster was restarted")
                _maybe_hard_fault(self.strategy, self.global_step.value())
                results = _execute(fetches, feed_dict, self._session)
                # a collective of this step missed its deadline / a peer was restarted while it
                # ran: the step's result is garbage (the watchdog aborted the communicator) --
                # recover BEFORE any hook (a checkpoint save!) observes it
                _comm_check()
                self._session.last_results = results
                rv = SessionRunValues(results)
                for h in self.hooks:
                    h.after_run(ctx, rv)
                break
            except Exception as e:
                # the step (or a hook observing it) failed: roll back to the latest checkpoint
                # (re-forming the cluster when a task died) and run the step again, like TF's
                # _RecoverableSession
                if not _recoverable(e):
                    raise
                attempts += 1
                if attempts > self.max_recovery_attempts:
                    raise
                # a recovery that itself hits a recoverable failure (the restarted task not up
                # yet, a peer dying mid-rejoin) is retried within the same attempt budget
                state = {}                # what this recovery already did (see _rejoin)
                while True:
                    try:
                        self._recover(e, state)
                        break
                    except Exception as e2:      # noqa: BLE001
                        # a TimeoutError already waited out the recovery budget: not retried
                        if isinstance(e2, TimeoutError) or not _recoverable(e2):
                            raise
                        attempts += 1
                        if attempts > self.max_recovery_attempts:
                            raise
                        print(f"[dtf] recovery failed ({type(e2).__name__}: {e2}); retrying "
                              f"({attempts}/{self.max_recovery_attempts})", flush=True)
                        e = e2
        if ctx.stop_requested:
            self._should_stop = True
        return results

    def run_step_fn(self, step_fn):
        return self.run(step_fn)

    def close(self):
        if self._closed:
            return
        try:
            for h in self.hooks:
                h.end(self._session)
        finally:
            self._closed = True
            client = getattr(self.strategy, "ps_client", None)
            if client is not None and client.params is not None:
                opt = self.scaffold.optimizer
                if opt is not None and getattr(opt, "space", None) is not None:
                    opt.synchronize_variables()     # the pipelined push in flight is answered
                _stop_client(client)
            if self._writer is not None:
                self._writer.close()

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        if exc_type is None or issubclass(exc_type, StopIteration):
            self.close()
            return exc_type is not None
        self._closed = True
        client = getattr(self.strategy, "ps_client", None)
        if client is not None and client.params is not None:
            # best effort: the failure being propagated may be the group itself (a recovery
            # that tore it down and could not re-form it) -- never mask it with the stop's error
            try:
                _stop_client(client)
            except Exception as e:      # noqa: BLE001
                print(f"[dtf] PS client stop after {exc_type.__name__} failed: {e!r}", flush=True)
        return False


def _stop_client(client):
    """Tell the parameter servers this worker is done -- only over a live process group (after
    a failed recovery the group may be torn down; there is nobody to tell then)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        client.stop()


class Supervisor:
    """``tf.train.Supervisor`` compat (``templates/00_mnist_replica.py:193-235``): chief
    initialises (``init_op`` callable) / restores from ``logdir``; others wait; the returned
    session supports ``run``."""

    def __init__(self, is_chief=True, logdir=None, init_op=None, local_init_op=None,
                 ready_for_local_init_op=None, recovery_wait_secs=1, global_step=None,
                 saver=None, model=None, optimizer=None, save_model_secs=600,
                 summary_writer=None, strategy=None):
        self.is_chief = is_chief
        self.logdir = logdir
        self.init_op = init_op
        self.local_init_op = local_init_op
        self.recovery_wait_secs = recovery_wait_secs
        self.global_step = global_step or gs_mod.get_or_create_global_step()
        self.model, self.optimizer, self.strategy = model, optimizer, strategy
        self.saver = saver
        self.save_model_secs = save_model_secs
        self._mts = None

    def prepare_or_wait_for_session(self, master="", config=None, wait_for_checkpoint=False,
                                    max_wait_secs=7200, start_standard_services=True):
        scaffold = Scaffold(self.model, self.optimizer, self.global_step, self.saver,
                            init_fn=(lambda s: self.init_op()) if callable(self.init_op) else None)
        self._mts = MonitoredTrainingSession(
            master, self.is_chief, self.logdir, scaffold, config=config,
            save_checkpoint_secs=self.save_model_secs if self.logdir else None,
            save_summaries_steps=None, log_step_count_steps=None, strategy=self.strategy)
        if callable(self.local_init_op):
            self.local_init_op()
        return self._mts

    def managed_session(self, master="", config=None):
        sess = self.prepare_or_wait_for_session(master, config)
        return sess

    def start_queue_runners(self, sess=None, queue_runners=None):
        return []

    def should_stop(self):
        return self._mts.should_stop() if self._mts else False

    def stop(self, threads=None, close_summary_writer=True):
        if self._mts is not None:
            self._mts.close()

    def request_stop(self, ex=None):
        if self._mts is not None:
            self._mts._should_stop = True


def wait_for_new_checkpoint(checkpoint_dir, last_checkpoint=None, seconds_to_sleep=1,
                            timeout=None):
    t0 = time.time()
    while True:
        ck = latest_checkpoint(checkpoint_dir)
        if ck and ck != last_checkpoint:
            return ck
        if timeout is not None and time.time() - t0 > timeout:
            return None
        time.sleep(seconds_to_sleep)


def default_checkpoint_dir():
    return os.path.join("/tmp", "train_logs")
