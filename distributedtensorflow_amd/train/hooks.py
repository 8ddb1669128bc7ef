"""SessionRunHook family (``tf.train.*Hook``) for :class:`MonitoredTrainingSession`.

Reference uses ``StopAtStepHook(last_step=1000)`` (``run_mnist_distributed.py:118-120``) and
relies on MTS's implicit checkpoint / summary saving (``templates/00_between…:40-46``).
"""
from __future__ import annotations

import math
import os
import time


class SessionRunArgs:
    def __init__(self, fetches=None, feed_dict=None, options=None):
        self.fetches, self.feed_dict, self.options = fetches, feed_dict, options


class SessionRunContext:
    def __init__(self, original_args, session):
        self.original_args = original_args
        self.session = session
        self._stop_requested = False

    def request_stop(self):
        self._stop_requested = True

    @property
    def stop_requested(self):
        return self._stop_requested


class SessionRunValues:
    def __init__(self, results, options=None, run_metadata=None):
        self.results, self.options, self.run_metadata = results, options, run_metadata


class SessionRunHook:
    def begin(self):
        pass

    def after_create_session(self, session, coord=None):
        pass

    def before_run(self, run_context):
        return None

    def after_run(self, run_context, run_values):
        pass

    def end(self, session):
        pass


def _gstep(session):
    gs = session.global_step
    return gs.value() if hasattr(gs, "value") else int(gs)


class StopAtStepHook(SessionRunHook):
    def __init__(self, num_steps=None, last_step=None):
        if (num_steps is None) == (last_step is None):
            raise ValueError("exactly one of num_steps / last_step must be given")
        self._num_steps, self._last_step = num_steps, last_step

    def after_create_session(self, session, coord=None):
        if self._last_step is None:
            self._last_step = _gstep(session) + self._num_steps

    def before_run(self, run_context):
        if _gstep(run_context.session) >= self._last_step:
            run_context.request_stop()

    def after_run(self, run_context, run_values):
        if _gstep(run_context.session) >= self._last_step:
            run_context.request_stop()

    @property
    def last_step(self):
        return self._last_step


class _Timer:
    def __init__(self, every_secs=None, every_steps=None):
        self.every_secs, self.every_steps = every_secs, every_steps
        self.last_time, self.last_step = None, None

    def should_trigger(self, step):
        if self.last_step is None:
            return True
        if self.every_steps is not None and step >= self.last_step + self.every_steps:
            return True
        if self.every_secs is not None and time.time() >= self.last_time + self.every_secs:
            return True
        return False

    def update(self, step):
        self.last_time, self.last_step = time.time(), step


class CheckpointSaverHook(SessionRunHook):
    def __init__(self, checkpoint_dir, save_secs=None, save_steps=None, saver=None,
                 checkpoint_basename="model.ckpt"):
        if save_secs is None and save_steps is None:
            save_secs = 600
        self.dir = checkpoint_dir
        self.timer = _Timer(save_secs, save_steps)
        self.saver = saver
        self.basename = checkpoint_basename
        self.saved = []

    def after_create_session(self, session, coord=None):
        self._save(session, _gstep(session))

    def after_run(self, run_context, run_values):
        step = _gstep(run_context.session)
        if self.timer.should_trigger(step):
            self._save(run_context.session, step)

    def end(self, session):
        step = _gstep(session)
        if self.timer.last_step != step:
            self._save(session, step)

    def _save(self, session, step):
        self.timer.update(step)
        saver = self.saver or session.saver
        if saver is None:
            return
        p = session.save_checkpoint(os.path.join(self.dir, self.basename), step, saver)
        if p is not None:          # None: a non-chief replica took part in a collective save
            self.saved.append(p)


class StepCounterHook(SessionRunHook):
    """Logs ``global_step/sec`` (and examples/sec given ``batch_size``) to a summary writer."""

    def __init__(self, every_n_steps=100, every_n_secs=None, output_dir=None,
                 summary_writer=None, batch_size=None):
        self.timer = _Timer(every_n_secs, every_n_steps)
        self.output_dir, self.writer = output_dir, summary_writer
        self.batch_size = batch_size
        self.last = None
        self.rates = []

    def after_run(self, run_context, run_values):
        step = _gstep(run_context.session)
        if self.timer.should_trigger(step):
            now = time.time()
            if self.last is not None:
                dt = now - self.last[1]
                if dt > 0 and step > self.last[0]:
                    rate = (step - self.last[0]) / dt
                    self.rates.append(rate)
                    vals = {"global_step/sec": rate}
                    if self.batch_size:
                        vals["examples/sec"] = rate * self.batch_size
                    w = self.writer or run_context.session.summary_writer
                    if w is not None:
                        w.add_scalars(vals, step)
            self.last = (step, now)
            self.timer.update(step)


class LoggingTensorHook(SessionRunHook):
    def __init__(self, tensors, every_n_iter=None, every_n_secs=None, formatter=None, at_end=False):
        self.tensors = tensors if isinstance(tensors, dict) else {str(t): t for t in tensors}
        self.timer = _Timer(every_n_secs, every_n_iter or (None if every_n_secs else 1))
        self.formatter = formatter
        self.at_end = at_end
        self.iter = 0
        self.lines = []

    def _fmt(self, values):
        if self.formatter:
            return self.formatter(values)
        return ", ".join(f"{k} = {v}" for k, v in values.items())

    def after_run(self, run_context, run_values):
        if self.timer.should_trigger(self.iter):
            named = _step_values(run_context, run_values)
            vals = {k: (float(v()) if callable(v) else
                        float(named[v]) if isinstance(v, str) else float(v))
                    for k, v in self.tensors.items()}
            line = self._fmt(vals)
            self.lines.append(line)
            print(line, flush=True)
            self.timer.update(self.iter)
        self.iter += 1


class SummarySaverHook(SessionRunHook):
    """Writes scalar summaries returned by the run (dict results) every N steps."""

    def __init__(self, save_steps=None, save_secs=None, output_dir=None, summary_writer=None,
                 scalars=None):
        self.timer = _Timer(save_secs, save_steps if save_steps or save_secs else 100)
        self.output_dir, self.writer, self.scalars = output_dir, summary_writer, scalars

    def after_run(self, run_context, run_values):
        step = _gstep(run_context.session)
        if not self.timer.should_trigger(step):
            return
        self.timer.update(step)
        vals = {k: float(v) for k, v in _step_values(run_context, run_values).items()
                if (self.scalars is None or k in self.scalars) and _is_number(v)}
        w = self.writer or run_context.session.summary_writer
        if vals and w is not None:
            w.add_scalars(vals, step)


class NanTensorHook(SessionRunHook):
    def __init__(self, loss_tensor=None, fail_on_nan_loss=True):
        self.loss, self.fail = loss_tensor, fail_on_nan_loss

    def after_run(self, run_context, run_values):
        if callable(self.loss):
            v = self.loss()
        else:
            v = _step_values(run_context, run_values).get(self.loss or "loss")
        if v is not None and not math.isfinite(float(v)):
            if self.fail:
                raise FloatingPointError("NaN loss during training.")
            run_context.request_stop()


class FinalOpsHook(SessionRunHook):
    def __init__(self, final_ops):
        self.final_ops = final_ops
        self.final_ops_values = None

    def end(self, session):
        self.final_ops_values = self.final_ops() if callable(self.final_ops) else self.final_ops


class FaultInjectionHook(SessionRunHook):
    """``DTF_FAULT_KILL_AT_STEP=rank:step`` — raise at a given step on a given rank (tests of the
    recover-from-checkpoint path)."""

    def __init__(self, spec=None, rank=0):
        spec = spec or os.environ.get("DTF_FAULT_KILL_AT_STEP", "")
        self.rank, self.step = (int(x) for x in spec.split(":")) if spec else (None, None)
        self.my_rank = rank
        self.fired = False

    def after_run(self, run_context, run_values):
        if self.step is not None and not self.fired and self.my_rank == self.rank and \
                _gstep(run_context.session) >= self.step:
            self.fired = True
            raise InjectedFault(f"injected fault at step {self.step}")


class InjectedFault(RuntimeError):
    pass


def _step_values(run_context, run_values):
    """Named values of the step: the dict returned by the train-op callable (whatever shape the
    fetch structure had), else the run results themselves when they are a dict."""
    named = getattr(run_context.session, "last_named", None)
    if named:
        return named
    res = run_values.results
    return res if isinstance(res, dict) else {}


def _is_number(v):
    try:
        float(v)
        return True
    except (TypeError, ValueError):
        return False
