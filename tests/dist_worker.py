"""One rank of a multi-process CPU (gloo) data-parallel run, launched by tests/test_distributed.py
exactly like torchrun would (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the env).

    python dist_worker.py <strategy> <out_dir> [key=value ...]

Each rank initialises its model with a DIFFERENT seed (the strategy must broadcast rank 0's
variables), trains on its own shard of a fixed global batch, and saves its final variables and
global step to ``out_dir/rank<r>.pt`` for the test to compare against a single-process run.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def global_batch(step, n=16):
    # explicit CPU: inside a GPU strategy's scope the default device is the GPU
    g = torch.Generator().manual_seed(1000 + step)
    return (torch.rand(n, 784, generator=g, device="cpu"),
            torch.randint(0, 10, (n,), generator=g, device="cpu"))


def make_optimizer(name):
    from distributedtensorflow_amd.optimizers import (AdamOptimizer, LAMBOptimizer,
                                                      MomentumOptimizer)
    if name == "lamb":
        return LAMBOptimizer(1e-3)
    return AdamOptimizer(1e-3) if name == "adam" else MomentumOptimizer(0.05, 0.9)


class _DirectDense(torch.autograd.Function):
    """Dense layer whose backward writes dW / db straight into the optimizer's flat gradient
    buffer and raises the parameter's readiness event itself -- the contract of the native
    kernels (ops/native.py _direct_grad / _grad_ready), reproduced on CPU so the bucketed
    all-reduce's handling of it is covered by gloo runs."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.params = (w, b)
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        grads = [dy.t() @ x, None if ctx.params[1] is None else dy.sum(0)]
        out = []
        for p, g in zip(ctx.params, grads):
            if g is not None and getattr(p, "_dtf_flat", False) and p.grad is not None:
                p.grad.add_(g)
                ready = getattr(p, "_dtf_grad_ready", None)
                if ready is not None:
                    ready()
                g = None
            out.append(g)
        return (dy @ w, *out)


def _direct_dense(x, w, b=None, relu=False):
    y = _DirectDense.apply(x, w, b)
    return torch.relu(y) if relu else y


def main():
    import faulthandler
    import signal
    faulthandler.register(signal.SIGUSR1)      # stack dump of a hung rank (tests' diagnostics)
    kind, out = sys.argv[1], sys.argv[2]
    kw = dict(a.split("=", 1) for a in sys.argv[3:])
    steps = int(kw.get("steps", 3))
    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import MnistCNN
    from distributedtensorflow_amd.parallel import (MirroredStrategy, MultiWorkerMirroredStrategy,
                                                    ParameterServerStrategy)
    if kind == "heartbeat":
        return heartbeat_probe(out)
    if kind == "hung_peer":
        return hung_peer_watchdog(out)
    if kind == "hang_mid_run":
        return hang_mid_run(out, kw)
    if kind == "mirrored_recovery":
        return mirrored_recovery(out, kw, steps)
    if kind == "resnet_gpu":
        return resnet_gpu_grads(out)
    if kind == "colocated_bert":
        return colocated_bert(out, kw, steps)
    if kind == "mirrored":
        strat = MirroredStrategy(bucket_mb=float(kw.get("bucket_mb", 64)),
                                 first_bucket_mb=float(kw.get("bucket_mb", 4)),
                                 compress_bf16=kw.get("bf16", "0") == "1",
                                 overlap=kw.get("overlap", "1") == "1")
    elif kind == "multiworker":
        strat = MultiWorkerMirroredStrategy()
    elif kind in ("colocated_ps", "colocated_ckpt"):
        strat = ParameterServerStrategy(num_ps=int(kw.get("num_ps", 1)),
                                        bucket_mb=float(kw.get("bucket_mb", 64)),
                                        first_bucket_mb=float(kw.get("bucket_mb", 4)),
                                        overlap_gather=kw.get("overlap", "1") == "1")
    else:
        raise SystemExit(f"unknown strategy {kind}")
    rank, world = strat.replica_id, strat.num_replicas_in_sync
    if kw.get("direct", "0") == "1":
        ops.dense = _direct_dense
    if kind == "colocated_ckpt":
        return checkpointed_run(strat, out, kw, steps)
    torch.manual_seed(17 + 101 * rank)
    with strat.scope():
        model = MnistCNN()
        opt = make_optimizer(kw.get("opt", "momentum"))
        gstep = dtf.train.get_or_create_global_step()
        opt.build(list(model.parameters()))
        per = 16 // world
        early = []
        for step in range(steps):
            x, y = global_batch(step)
            x, y = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
            loss = ops.sparse_softmax_cross_entropy(model(x), y)
            opt.minimize(loss, global_step=gstep)
            st = getattr(opt._reducer, "stats", None)
            if st is not None:
                early.append((st.last_early, st.n_buckets))
        mean_loss = float(strat.reduce(dtf.distribute.ReduceOp.MEAN, loss.detach()))
        fps = dtf.distribute.check_replicas_consistent(opt)      # raises if replicas diverged
        red = opt._reducer
        agreement = None
        if hasattr(red, "plan") and world > 1:
            from distributedtensorflow_amd.parallel import verify_bucket_agreement
            agreement = verify_bucket_agreement(red)      # raises on a plan / order mismatch
    torch.save({"state": {k: v.detach().clone() for k, v in model.state_dict().items()},
                "global_step": gstep.value(), "world": world, "mean_loss": mean_loss,
                "fingerprints": fps, "early_launches": early,
                "sharded": getattr(opt._reducer, "sharded", None),
                "reducer": type(opt._reducer).__name__,
                "plan": red.plan() if hasattr(red, "plan") else None,
                "order": list(getattr(red, "last_order", ())),
                "ranges": [list(r) for r in getattr(red, "ranges", [])],
                "agreement": agreement},
               os.path.join(out, f"rank{rank}.pt"))
    strat.barrier()


def colocated_bert(out, kw, steps):
    """A tiny BERT (every dense layer, the fused bias + GELU + dense FFN op, LayerNorms,
    embeddings) under the sharded colocated parameter server with many buckets: with the
    overlapped all-gather pull, every op that reads a variable must wait for that variable's
    bucket (ops parameter fence).  The test compares the run with overlap on to overlap off."""
    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models.bert import BertConfig, BertForPreTraining
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import ParameterServerStrategy
    strat = ParameterServerStrategy(num_ps=2, bucket_mb=0.02, first_bucket_mb=0.02,
                                    overlap_gather=kw.get("overlap", "1") == "1")
    rank, world = strat.replica_id, strat.num_replicas_in_sync
    torch.manual_seed(31 + 7 * rank)            # rank 0's variables must win the broadcast
    cfg = BertConfig(vocab_size=200, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                     intermediate_size=256, max_position_embeddings=32, hidden_dropout_prob=0.0,
                     attention_probs_dropout_prob=0.0)
    with strat.scope():
        model = BertForPreTraining(cfg)
        opt = MomentumOptimizer(0.05, 0.9)
        gstep = dtf.train.get_or_create_global_step()
        opt.build(list(model.parameters()))
        for step in range(steps):
            g = torch.Generator().manual_seed(500 + 10 * step + rank)
            B, S, P = 2, 16, 4
            ids = torch.randint(0, 200, (B, S), generator=g, device="cpu")
            tt = torch.zeros(B, S, dtype=torch.long)
            am = torch.ones(B, S)
            pos = torch.randint(0, S, (B, P), generator=g, device="cpu")
            lab = torch.randint(0, 200, (B, P), generator=g, device="cpu")
            w = torch.ones(B, P)
            loss = model(ids, tt, am, pos, lab, w)
            opt.minimize(loss, global_step=gstep)
        fps = dtf.distribute.check_replicas_consistent(opt)      # raises if replicas diverged
    torch.save({"state": {k: v.detach().clone() for k, v in model.state_dict().items()},
                "fingerprints": fps, "sharded": getattr(opt._reducer, "sharded", None),
                "loss": float(loss.detach())}, os.path.join(out, f"rank{rank}.pt"))
    strat.barrier()
    # results are on disk: leave without the interpreter teardown, where gloo's threads behind the
    # still-registered overlapped gathers intermittently hit std::terminate (exit -6)
    sys.stdout.flush()
    os._exit(0)


def checkpointed_run(strat, out, kw, steps):
    """MonitoredTrainingSession on every rank of a colocated (sharded) parameter server with a
    step-triggered checkpoint: the save is collective (slot shards gathered from their owners),
    the chief writes it.  A second session then restores it on the chief and must hand the
    restored state to every rank."""
    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import MnistCNN
    rank, world = strat.replica_id, strat.num_replicas_in_sync
    torch.manual_seed(17 + 101 * rank)
    ckpt = os.path.join(out, "ckpt")
    per = 16 // world
    with strat.scope():
        model = MnistCNN()
        opt = make_optimizer(kw.get("opt", "adam"))
        gstep = dtf.train.get_or_create_global_step()
        opt.build(list(model.parameters()))

        def step_fn(step):
            x, y = global_batch(step)
            x, y = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
            opt.minimize(ops.sparse_softmax_cross_entropy(model(x), y), global_step=gstep)

        with dtf.train.MonitoredTrainingSession(
                is_chief=rank == 0, checkpoint_dir=ckpt, save_checkpoint_steps=steps,
                save_summaries_steps=None, log_step_count_steps=None, model=model,
                optimizer=opt, global_step=gstep, strategy=strat) as sess:
            while gstep.value() < steps:
                s = gstep.value()
                sess.run(lambda: step_fn(s))
        opt.synchronize_variables()
        # a fresh session on perturbed variables: the chief restores, everyone must follow
        with torch.no_grad():
            opt.space.master.add_(1.0 + rank)
            opt.space.refresh_shadow()
            for t in opt.state_tensors():
                t.mul_(3.0 + rank)
        opt.iterations = 99 + rank
        gstep.assign(7 * (rank + 1))
        sess2 = dtf.train.MonitoredTrainingSession(
            is_chief=rank == 0, checkpoint_dir=ckpt, save_checkpoint_steps=None,
            save_checkpoint_secs=None, save_summaries_steps=None, log_step_count_steps=None,
            model=model, optimizer=opt, global_step=gstep, strategy=strat)
        restored = {"master": opt.space.master.detach().clone(),
                    "slots": [t.detach().clone() for t in opt.state_tensors()],
                    "iterations": opt.iterations, "global_step": gstep.value()}
        sess2.close()
    torch.save({"restored": restored, "sharded": getattr(opt._reducer, "sharded", None)},
               os.path.join(out, f"rank{rank}.pt"))
    strat.barrier()


def mirrored_recovery(out, kw, steps):
    """A rank of a MirroredStrategy world under launch_collective, trained with a
    MonitoredTrainingSession that checkpoints every ``save`` steps.  With
    DTF_FAULT_SIGKILL=rank:1@k rank 1 dies mid-run; the launcher restarts it, rank 0 re-forms the
    world in the new epoch, the chief's latest checkpoint is restored and broadcast, and both
    reach ``steps`` with identical variables."""
    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import MnistCNN
    from distributedtensorflow_amd.parallel import MirroredStrategy, ParameterServerStrategy
    strat = (ParameterServerStrategy(num_ps=2) if kw.get("strategy") == "ps"
             else MirroredStrategy())
    rank, world = strat.replica_id, strat.num_replicas_in_sync
    torch.manual_seed(17 + 101 * rank)
    per = 16 // world
    with strat.scope():
        model = MnistCNN()
        opt = make_optimizer(kw.get("opt", "momentum"))
        gstep = dtf.train.get_or_create_global_step()
        opt.build(list(model.parameters()))

        def step_fn(step):
            x, y = global_batch(step)
            x, y = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
            x, y = x.to(strat.device), y.to(strat.device)
            opt.minimize(ops.sparse_softmax_cross_entropy(model(x), y), global_step=gstep)

        sess = dtf.train.MonitoredTrainingSession(
            is_chief=rank == 0, checkpoint_dir=os.path.join(out, "ckpt"),
            save_checkpoint_steps=int(kw.get("save", 3)), save_summaries_steps=None,
            log_step_count_steps=None, model=model, optimizer=opt, global_step=gstep,
            strategy=strat)
        with sess:
            while gstep.value() < steps:
                s = gstep.value()
                sess.run(lambda: step_fn(s))
                print(f"rank {rank} step {gstep.value()}", flush=True)
        fps = dtf.distribute.check_replicas_consistent(opt)
    torch.save({"state": {k: v.detach().cpu().clone() for k, v in model.state_dict().items()},
                "master": opt.space.master.detach().cpu().clone(),
                "comm": getattr(getattr(opt._reducer, "comm", None), "kind", None),
                "reducer": type(opt._reducer).__name__,
                "global_step": gstep.value(), "recoveries": sess.recoveries,
                "fingerprints": fps, "restart": int(os.environ.get("DTF_RESTART_COUNT", "0"))},
               os.path.join(out, f"rank{rank}.pt"))
    strat.barrier()


def resnet_batch():
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 64, 64, 3, generator=g, device="cpu").to(torch.bfloat16)
    return x, torch.randint(0, 1000, (4,), generator=g, device="cpu")


def resnet_gpu_grads(out):
    """Two ranks sharing one GPU over gloo: ResNet-50 gradients through the native kernels
    (direct flat-buffer writes, lazy residual gradients, bucketed all-reduce).  Saves the
    all-reduced (summed) gradient buffer and the broadcast initial variables."""
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import resnet50
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import MirroredStrategy
    strat = MirroredStrategy(bucket_mb=8, first_bucket_mb=1, backend="gloo")
    rank = strat.replica_id
    torch.manual_seed(17 + 101 * rank)
    with strat.scope():
        model = resnet50().cuda()
        opt = MomentumOptimizer(0.1, 0.9)
        opt.build(list(model.parameters()))
        init = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
        x, y = resnet_batch()
        x, y = x[2 * rank:2 * rank + 2].cuda(), y[2 * rank:2 * rank + 2].cuda()
        loss = ops.sparse_softmax_cross_entropy(model(x), y)
        opt.compute_gradients(loss, list(model.parameters()))
        torch.cuda.synchronize()
        torch.save({"init": init, "grad": opt.space.grad.cpu().clone(),
                    "order": [n for n, p in model.named_parameters()]},
                   os.path.join(out, f"rank{rank}.pt"))
    strat.barrier()


def hang_mid_run(out, kw):
    """A 2-rank MirroredStrategy world under launch_collective WITHOUT restarts: rank 1 hangs
    (alive, stops stepping) at global step ``at``.  Rank 0's collective must fail within
    DTF_COMM_TIMEOUT_S and end its process non-zero; the launcher then stops rank 1 -- the job
    ends loudly instead of hanging."""
    import time

    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import MnistCNN
    from distributedtensorflow_amd.parallel import MirroredStrategy
    strat = MirroredStrategy()
    rank = strat.replica_id
    at = int(kw.get("at", 4))
    torch.manual_seed(3)
    with strat.scope():
        model = MnistCNN()
        opt = make_optimizer("momentum")
        gstep = dtf.train.get_or_create_global_step()
        opt.build(list(model.parameters()))
        sess = dtf.train.MonitoredTrainingSession(
            is_chief=rank == 0, checkpoint_dir=None, save_checkpoint_secs=None,
            save_summaries_steps=None, log_step_count_steps=None, model=model, optimizer=opt,
            global_step=gstep, strategy=strat)
        with sess:
            while gstep.value() < 50:
                s = gstep.value()
                if rank == 1 and s == at:
                    print("rank 1 hangs", flush=True)
                    time.sleep(3600)
                x, y = global_batch(s)
                x, y = x[rank * 8:(rank + 1) * 8], y[rank * 8:(rank + 1) * 8]
                sess.run(lambda: opt.minimize(ops.sparse_softmax_cross_entropy(model(x), y),
                                              global_step=gstep))
                print(f"rank {rank} step {gstep.value()}", flush=True)


def hung_peer_watchdog(out):
    """Rank 1 hangs (alive, never enters the collective); rank 0's all-reduce must be flagged by
    the collective watchdog within DTF_COMM_TIMEOUT_S and surface as CommError -- not block."""
    import json
    import time

    from distributedtensorflow_amd.parallel import init_process_group_from_env
    from distributedtensorflow_amd.parallel.comm import C10dComm
    from distributedtensorflow_amd.parallel.strategy import CommError
    from distributedtensorflow_amd.parallel.watchdog import get_watchdog
    init_process_group_from_env("gloo")
    import torch.distributed as dist
    rank = dist.get_rank()
    dist.barrier()
    if rank == 1:
        time.sleep(12.0)
        os._exit(0)
    comm = C10dComm()
    wd = get_watchdog()
    t0 = time.time()
    comm.all_reduce(torch.ones(1024))
    tripped = wd.wait_tripped(15.0)
    after = time.time() - t0
    err = None
    try:
        comm.all_reduce(torch.ones(4))
    except CommError as e:
        err = str(e)
    with open(os.path.join(out, "wd.json"), "w") as f:
        json.dump({"tripped": tripped, "after_s": after, "error": err,
                   "reason": wd.failed}, f)
    os._exit(0)


def heartbeat_probe(out):
    """rank 1 stops beating (a hung / dead peer); rank 0 must notice it and no one else."""
    import json
    import time

    from distributedtensorflow_amd.parallel import Heartbeat, init_process_group_from_env
    init_process_group_from_env("gloo")
    import torch.distributed as dist
    rank = dist.get_rank()
    hb = Heartbeat(interval_s=0.2, timeout_s=1.5).start()
    dist.barrier()
    if rank == 1:
        hb.stop()                       # simulated failure: heartbeats stop, process stays
        time.sleep(4.0)
    else:
        t0 = time.time()
        while 1 not in hb.failed_peers and time.time() - t0 < 10:
            time.sleep(0.1)
        with open(os.path.join(out, "hb.json"), "w") as f:
            json.dump({"failed": sorted(hb.failed_peers), "after_s": time.time() - t0}, f)
        hb.stop()
    dist.barrier()


if __name__ == "__main__":
    main()
