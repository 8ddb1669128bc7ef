"""MonitoredTrainingSession + hooks + TF-V2 Saver on CPU (reference
``run_mnist_distributed.py:118-161``, ``templates/00_between…:40-52``):
stop-at-step, periodic checkpoints in TF layout, restore-and-continue, fault recovery,
Supervisor, SavedModel export."""
import os

import numpy as np
import pytest
import torch

from distributedtensorflow_amd import ops
from distributedtensorflow_amd.io.bundle import BundleReader
from distributedtensorflow_amd.models import MnistCNN
from distributedtensorflow_amd.optimizers import AdamOptimizer
from distributedtensorflow_amd.parallel import OneDeviceStrategy
from distributedtensorflow_amd.summary.events import read_scalars
from distributedtensorflow_amd.train import (CheckpointSaverHook, FaultInjectionHook,
                                             LoggingTensorHook, MonitoredTrainingSession,
                                             NanTensorHook, Saver, StopAtStepHook, Supervisor,
                                             get_checkpoint_state, latest_checkpoint,
                                             list_variables, load_saved_model_variables,
                                             load_variable, reset_global_step,
                                             save_saved_model)
from distributedtensorflow_amd.train import global_step as gs_mod


@pytest.fixture(autouse=True)
def _fresh_global_step():
    reset_global_step()
    yield
    reset_global_step()


def _setup(seed=0):
    torch.manual_seed(seed)
    strat = OneDeviceStrategy("cpu")
    with strat.scope():
        model = MnistCNN()
        opt = AdamOptimizer(5e-4)
        gstep = gs_mod.get_or_create_global_step()
        opt.build(list(model.parameters()))
    g = torch.Generator().manual_seed(7)
    x = torch.rand(16, 784, generator=g)
    y = torch.randint(0, 10, (16,), generator=g)

    def train_op():
        loss = ops.sparse_softmax_cross_entropy(model(x), y)
        opt.minimize(loss, global_step=gstep)
        return {"loss": loss}
    return strat, model, opt, gstep, train_op


def test_stop_at_step_checkpoints_and_summaries(tmp_path):
    ck = str(tmp_path / "ck")
    strat, model, opt, gstep, train_op = _setup()
    losses = []
    with MonitoredTrainingSession(checkpoint_dir=ck, hooks=[StopAtStepHook(last_step=6)],
                                  save_checkpoint_steps=3, save_summaries_steps=2,
                                  log_step_count_steps=2, model=model, optimizer=opt,
                                  global_step=gstep, strategy=strat) as sess:
        while not sess.should_stop():
            out = sess.run([train_op, "loss", gstep])
            if out is None:
                break
            losses.append(out[1])
            assert out[2] == len(losses)
    assert gstep.value() == 6 and len(losses) == 6
    state = get_checkpoint_state(ck)
    assert os.path.basename(state.model_checkpoint_path) == "model.ckpt-6"
    names = dict(list_variables(ck))
    # TF layouts: HWIO conv kernels, [in, out] dense kernels, Adam slots, beta powers
    assert names["conv2d/kernel"] == [5, 5, 1, 32]
    assert names["dense/kernel"] == [3136, 1024]
    assert names["conv2d/kernel/Adam_1"] == [5, 5, 1, 32]
    assert names["global_step"] == []
    assert float(load_variable(ck, "beta1_power")) == pytest.approx(0.9 ** 7)
    k = load_variable(ck, "conv2d/kernel")
    np.testing.assert_allclose(k, model.conv1.kernel.detach().permute(1, 2, 3, 0).numpy())
    assert os.path.exists(latest_checkpoint(ck) + ".meta")
    sc = read_scalars(ck)
    assert "loss" in sc and "global_step/sec" in sc


def test_restore_continues_from_checkpoint(tmp_path):
    ck = str(tmp_path / "ck")
    strat, model, opt, gstep, train_op = _setup(seed=0)
    with MonitoredTrainingSession(checkpoint_dir=ck, hooks=[StopAtStepHook(last_step=4)],
                                  save_summaries_steps=None, log_step_count_steps=None,
                                  model=model, optimizer=opt, global_step=gstep,
                                  strategy=strat) as sess:
        while not sess.should_stop():
            sess.run(train_op)
    ref_state = {n: t.detach().clone() for n, t in model.state_dict().items()}
    # a brand-new process-equivalent: different init, restored by the chief session
    reset_global_step()
    strat2, model2, opt2, gstep2, train_op2 = _setup(seed=123)
    with MonitoredTrainingSession(checkpoint_dir=ck, hooks=[StopAtStepHook(num_steps=2)],
                                  save_summaries_steps=None, log_step_count_steps=None,
                                  model=model2, optimizer=opt2, global_step=gstep2,
                                  strategy=strat2) as sess:
        assert gstep2.value() == 4 and opt2.iterations == 4
        for n, t in model2.state_dict().items():
            torch.testing.assert_close(t, ref_state[n])
        torch.testing.assert_close(opt2.slots[0].buf, opt.slots[0].buf)
        while not sess.should_stop():
            sess.run(train_op2)
    assert gstep2.value() == 6
    # identical to continuing the original run for two more steps
    for _ in range(2):
        train_op()
    for n, t in model2.state_dict().items():
        torch.testing.assert_close(t, model.state_dict()[n])


def test_fault_injection_recovers_from_checkpoint(tmp_path):
    ck = str(tmp_path / "ck")
    strat, model, opt, gstep, train_op = _setup()
    fault = FaultInjectionHook("0:5", rank=0)
    with MonitoredTrainingSession(checkpoint_dir=ck,
                                  hooks=[StopAtStepHook(last_step=8), fault],
                                  save_checkpoint_steps=2, save_summaries_steps=None,
                                  log_step_count_steps=None, model=model, optimizer=opt,
                                  global_step=gstep, strategy=strat) as sess:
        steps = []
        while not sess.should_stop():
            sess.run(train_op)
            steps.append(gstep.value())
    assert fault.fired
    # step 5 failed -> rolled back to the step-4 checkpoint and re-ran
    assert steps[:4] == [1, 2, 3, 4] and steps[4] == 5 and gstep.value() == 8


def test_failed_recovery_is_retried_within_the_attempt_budget(tmp_path):
    """A recovery that itself hits a recoverable failure (the restarted task not up yet) is
    retried within max_recovery_attempts instead of escaping run()."""
    from distributedtensorflow_amd.train.session import InjectedFault
    ck = str(tmp_path / "ck")
    strat, model, opt, gstep, train_op = _setup()
    fault = FaultInjectionHook("0:5", rank=0)
    with MonitoredTrainingSession(checkpoint_dir=ck,
                                  hooks=[StopAtStepHook(last_step=8), fault],
                                  save_checkpoint_steps=2, save_summaries_steps=None,
                                  log_step_count_steps=None, model=model, optimizer=opt,
                                  global_step=gstep, strategy=strat) as sess:
        real, calls = sess._recover, []

        def flaky(exc=None, state=None):
            calls.append(type(exc).__name__)
            if len(calls) == 1:
                raise InjectedFault("recovery interrupted")
            return real(exc, state)
        sess._recover = flaky
        while not sess.should_stop():
            sess.run(train_op)
    assert fault.fired and len(calls) == 2 and gstep.value() == 8


def test_recovery_retry_resumes_after_the_rejoin():
    """A recovery whose post-rejoin phase fails (here the synchronous world's post-restore sync)
    is retried WITHOUT re-forming the cluster again: recover_cluster would wait for an epoch
    after the one just joined, which only comes if another task is restarted.  Only a cluster
    that moved on meanwhile (cluster_changed) is re-joined.  One recovery is counted once."""
    from distributedtensorflow_amd.train.session import MonitoredTrainingSession as MTS

    class _Strat:
        collective = True

        def __init__(self):
            self.rejoins, self.syncs, self.moved = 0, 0, False

        def recover_cluster(self, optimizer=None):
            self.rejoins += 1
            self.moved = False
            return self.rejoins

        def cluster_changed(self):
            return self.moved

        def sync_after_restore(self, optimizer, global_step, restored=False):
            self.syncs += 1
            if self.syncs == 1:
                raise ConnectionError("peer died mid-rejoin")

    class _Scaffold:
        optimizer = saver = None

        class global_step:
            @staticmethod
            def value():
                return 7

    sess = MTS.__new__(MTS)
    sess.strategy, sess.scaffold, sess.hooks = _Strat(), _Scaffold(), []
    sess.checkpoint_dir, sess.is_chief, sess._session, sess.recoveries = None, True, None, 0
    state = {}
    with pytest.raises(ConnectionError):
        sess._recover(ConnectionError("peer died"), state)
    sess._recover(ConnectionError("peer died"), state)       # the retry
    assert sess.strategy.rejoins == 1 and sess.strategy.syncs == 2 and sess.recoveries == 1
    # the cluster moved to a newer epoch before the retry: that one is joined
    state = {}
    sess.strategy.syncs = 0
    with pytest.raises(ConnectionError):
        sess._recover(ConnectionError("peer died"), state)
    sess.strategy.moved = True
    sess._recover(ConnectionError("peer died"), state)
    assert sess.strategy.rejoins == 3 and sess.recoveries == 2


def test_exit_never_masks_the_failure_with_the_ps_stop():
    """__exit__ on an exception: the PS client's stop is best effort (after a failed recovery
    the process group may be gone) -- the original exception propagates."""
    strat, model, opt, gstep, train_op = _setup()

    class _Client:
        params = [1]

        def stop(self):
            raise ValueError("Default process group has not been initialized")
    with pytest.raises(RuntimeError, match="primary"):
        with MonitoredTrainingSession(model=model, optimizer=opt, global_step=gstep,
                                      strategy=strat, save_summaries_steps=None,
                                      log_step_count_steps=None) as sess:
            sess.strategy.ps_client = _Client()
            raise RuntimeError("primary failure")


def test_nan_and_logging_hooks(tmp_path, capsys):
    strat, model, opt, gstep, train_op = _setup()
    hook = LoggingTensorHook(["loss"], every_n_iter=1)
    with MonitoredTrainingSession(hooks=[StopAtStepHook(last_step=2), hook, NanTensorHook()],
                                  model=model, optimizer=opt, global_step=gstep,
                                  strategy=strat) as sess:
        while not sess.should_stop():
            sess.run(train_op)
    assert "loss" in capsys.readouterr().out

    def bad_op():
        return {"loss": torch.tensor(float("nan"))}
    with pytest.raises(Exception):
        with MonitoredTrainingSession(hooks=[NanTensorHook()], model=model, optimizer=opt,
                                      global_step=gstep, strategy=strat) as sess:
            sess.run(bad_op)


def test_supervisor_and_saver_max_to_keep(tmp_path):
    logdir = str(tmp_path / "sv")
    strat, model, opt, gstep, train_op = _setup()
    inits = []
    sv = Supervisor(is_chief=True, logdir=logdir, init_op=lambda: inits.append(1),
                    recovery_wait_secs=1, global_step=gstep, model=model, optimizer=opt,
                    strategy=strat)
    sess = sv.prepare_or_wait_for_session("")
    for _ in range(3):
        sess.run(train_op)
    sv.stop()
    assert inits == [1] and gstep.value() == 3
    assert latest_checkpoint(logdir).endswith("model.ckpt-3")
    saver = Saver(model=model, optimizer=opt, global_step=gstep, max_to_keep=2)
    for s in (10, 11, 12):
        saver.save(None, str(tmp_path / "keep" / "m"), global_step=s)
    kept = sorted(f for f in os.listdir(tmp_path / "keep") if f.endswith(".index"))
    assert kept == ["m-11.index", "m-12.index"]
    st = get_checkpoint_state(str(tmp_path / "keep"))
    assert [os.path.basename(p) for p in st.all_model_checkpoint_paths] == ["m-11", "m-12"]


def test_sharded_saver_and_saved_model(tmp_path):
    strat, model, opt, gstep, train_op = _setup()
    train_op()
    saver = Saver(model=model, optimizer=opt, global_step=gstep, num_shards=3)
    p = saver.save(None, str(tmp_path / "s" / "model.ckpt"), global_step=gstep)
    assert os.path.exists(p + ".data-00002-of-00003")
    r = BundleReader(p)
    assert "dense_1/bias/Adam" in r.keys()
    exp = save_saved_model(str(tmp_path / "export"), model)
    assert os.path.exists(os.path.join(exp, "saved_model.pb"))
    with strat.scope():
        m2 = MnistCNN()
    load_saved_model_variables(exp, m2)
    for (n, a), (_, b) in zip(model.state_dict().items(), m2.state_dict().items()):
        torch.testing.assert_close(a, b)
