"""``train.py`` — one CLI for every model x strategy combination.

Keeps the reference's flags and adds strategy selection:

    # reference mode: between-graph parameter-server cluster (run_mnist_distributed.py:164-182)
    python train.py --job_name=ps     --task_index=0 [--config config.json]
    python train.py --job_name=worker --task_index=0 [--sync_replicas]
    #   ... or the template's comma lists (templates/00_mnist_replica.py:80-83)
    python train.py --job_name=worker --task_index=1 --ps_hosts=h:2222 --worker_hosts=h:2223,h:2224

    # tf.distribute-style strategies (one process per GPU; --num_gpus N spawns them via
    # torch.distributed.run on 127.0.0.1, or launch under torchrun / TF_CONFIG yourself)
    python train.py --model mnist_mlp --strategy onedevice --device cpu      # BASELINE config 1
    python train.py --model resnet50 --strategy mirrored --num_gpus 8        # configs 2 / 3
    python train.py --model resnet50 --strategy ps --num_ps 1 --num_gpus 8   # config 4
    python train.py --model bert_base --strategy multiworker --num_gpus 8    # config 5

The chief prints the reference's ``Worker (i): loss = x.xx (global step: n)`` line every
``--log_every`` steps and writes ``Global Step`` / ``Loss`` TensorBoard scalars under
``--log_dir/<timestamp>`` (``run_mnist_distributed.py:136-159``); ``--checkpoint_dir`` enables TF-V2
checkpoints + restore-on-restart through MonitoredTrainingSession.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import subprocess
import sys
import time

MODELS = ("mnist_cnn", "mnist_mlp", "resnet50", "resnet101", "resnet152", "bert_base",
          "bert_large")
STRATEGIES = ("onedevice", "mirrored", "multiworker", "ps")


def build_parser():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    # reference flags (run_mnist_distributed.py:167-180, templates/00_mnist_replica.py:49-84)
    p.add_argument("--job_name", default=None, help="ps | worker (between-graph cluster mode)")
    p.add_argument("--task_index", type=int, default=0)
    p.add_argument("--config", default="config.json", help="cluster JSON (ps / workers)")
    p.add_argument("--ps_hosts", default=None)
    p.add_argument("--worker_hosts", default=None)
    p.add_argument("--existing_servers", action="store_true",
                   help="attach to an already running cluster rendezvous (template R18)")
    p.add_argument("--sync_replicas", action="store_true")
    p.add_argument("--replicas_to_aggregate", type=int, default=None)
    p.add_argument("--num_gpus", type=int, default=None,
                   help="GPUs on this node (one process each); 0 = CPU")
    p.add_argument("--data_dir", default="/tmp/data/")
    p.add_argument("--download_only", action="store_true")
    p.add_argument("--hidden_units", type=int, default=100)
    p.add_argument("--train_steps", "--max_steps", dest="max_steps", type=int, default=1000)
    p.add_argument("--batch_size", type=int, default=None, help="per-replica batch")
    p.add_argument("--learning_rate", type=float, default=None)
    # framework flags
    p.add_argument("--model", choices=MODELS, default="mnist_cnn")
    p.add_argument("--strategy", choices=STRATEGIES, default=None)
    p.add_argument("--device", choices=("auto", "cpu", "gpu"), default="auto")
    p.add_argument("--optimizer", choices=("adam", "adagrad", "momentum", "sgd", "lamb"),
                   default=None)
    p.add_argument("--num_ps", type=int, default=None, help="colocated PS owners (strategy ps)")
    p.add_argument("--variable_placement", choices=("balanced", "round_robin"),
                   default="balanced")
    p.add_argument("--bucket_mb", type=float, default=64)
    p.add_argument("--image_size", type=int, default=224)
    p.add_argument("--seq_len", type=int, default=128)
    p.add_argument("--log_dir", default="/tmp/distributed_logs")
    p.add_argument("--log_every", type=int, default=1)
    p.add_argument("--checkpoint_dir", default=None)
    p.add_argument("--save_checkpoint_steps", type=int, default=None)
    p.add_argument("--save_checkpoint_secs", type=int, default=600)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--eval", action="store_true", help="evaluate on the MNIST test set at the end")
    return p


DEFAULTS = {   # (batch, optimizer, learning rate) per model
    "mnist_cnn": (128, "adam", 5e-4),          # run_mnist_distributed.py:77,116
    "mnist_mlp": (100, "adam", 0.01),          # templates/00_mnist_replica.py:66-69
    "resnet50": (256, "momentum", 0.1),
    "resnet101": (256, "momentum", 0.1),
    "resnet152": (256, "momentum", 0.1),
    "bert_base": (128, "lamb", 1e-3),
    "bert_large": (64, "lamb", 1e-3),
}


def _spawn_local(args, argv):
    """--num_gpus N > 1 without a torch.distributed env: start N ranks as CHILD processes
    (torch.distributed.run on 127.0.0.1) and return their exit code.  Nothing in this parent
    process touches the GPU."""
    from .cluster.launcher import free_ports
    port = free_ports(1)[0]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.num_gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(sys.argv[0]), *argv]
    return subprocess.call(cmd)


def _make_optimizer(name, lr, model_name, batch_global):
    from . import optimizers as O
    from .optimizers.optimizers import cosine_decay, polynomial_decay
    if name == "adam":
        return O.AdamOptimizer(lr)
    if name == "adagrad":
        return O.AdagradOptimizer(lr)
    if name == "sgd":
        return O.GradientDescentOptimizer(lr)
    if name == "momentum":
        if model_name.startswith("resnet"):
            return O.MomentumOptimizer(cosine_decay(lr * batch_global / 256, 90 * 5000,
                                                    warmup_steps=500), 0.9, weight_decay=1e-4)
        return O.MomentumOptimizer(lr, 0.9)
    if name == "lamb":
        return O.LAMBOptimizer(polynomial_decay(lr, 10000, warmup_steps=100), weight_decay=0.01)
    raise ValueError(name)


def _cluster_from_args(args):
    from .cluster import ClusterSpec, Config
    from .cluster.spec import from_flags
    if args.ps_hosts or args.worker_hosts:
        return from_flags(args.ps_hosts or "", args.worker_hosts or "")
    ps, workers = Config(args.config).get_ps_and_worker_hosts()
    return ClusterSpec({"ps": list(ps), "worker": list(workers)})


def run(args):
    import torch

    import distributedtensorflow_amd as dtf
    from . import ops
    from .parallel import (MirroredStrategy, MultiWorkerMirroredStrategy, OneDeviceStrategy,
                           ParameterServerStrategy)
    from .summary import logger
    from .train import (ConfigProto, MonitoredTrainingSession, StopAtStepHook,
                        get_or_create_global_step)

    print("run main with args =", args, flush=True)
    batch, opt_name, lr = DEFAULTS[args.model]
    batch = args.batch_size or batch
    opt_name = args.optimizer or opt_name
    lr = args.learning_rate if args.learning_rate is not None else lr
    want_gpu = (args.device == "gpu" or
                (args.device == "auto" and torch.cuda.is_available() and args.num_gpus != 0))

    server = None
    if args.job_name:                                   # ---- between-graph PS cluster
        from .cluster import Server
        cluster = _cluster_from_args(args)
        server = Server(cluster, job_name=args.job_name, task_index=args.task_index)
        if args.job_name == "ps":
            print("Started Parameter Server ...", flush=True)
            stats = server.join()
            print("Close Parameter Server ...", stats, flush=True)
            if not stats.get("interrupted"):
                server.shutdown()
            return 0
        if want_gpu:
            device = torch.device("cuda", args.task_index % torch.cuda.device_count())
        else:
            device = torch.device("cpu")
        strategy = ParameterServerStrategy(server=server, sync=args.sync_replicas,
                                           replicas_to_aggregate=args.replicas_to_aggregate,
                                           variable_placement=args.variable_placement,
                                           device=device)
    else:                                               # ---- tf.distribute strategies
        name = args.strategy or ("mirrored" if want_gpu else "onedevice")
        if name == "onedevice":
            strategy = OneDeviceStrategy("/gpu:0" if want_gpu else "/cpu:0")
        elif name == "mirrored":
            strategy = MirroredStrategy(bucket_mb=args.bucket_mb)
        elif name == "multiworker":
            strategy = MultiWorkerMirroredStrategy(bucket_mb=args.bucket_mb)
        else:
            strategy = ParameterServerStrategy(num_ps=args.num_ps,
                                               variable_placement=args.variable_placement)
        device = strategy.device
    rid, nrep = strategy.replica_id, strategy.num_replicas_in_sync
    is_chief = strategy.is_chief
    torch.manual_seed(args.seed)
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32

    # ---- data + model
    if args.model.startswith("mnist"):
        from .data import DeviceArrayDataset, mnist
        imgs, labels = mnist.load_arrays(args.data_dir, "train")
        if args.download_only:
            mnist.load_arrays(args.data_dir, "test")
            return 0
        shards = nrep if server is None else 1
        data = DeviceArrayDataset(imgs, labels, batch, device, dtype, shuffle=False,
                                  num_shards=shards, shard_index=rid if shards > 1 else 0)
    elif args.model.startswith("resnet"):
        from .data import SyntheticImageNet
        data = SyntheticImageNet(batch, args.image_size, device=device, dtype=dtype,
                                 seed=1234 + rid)
    else:
        from .data import SyntheticMLM
        data = SyntheticMLM(batch, args.seq_len, device=device, seed=1234 + rid)

    with strategy.scope():
        if args.model == "mnist_cnn":
            model = dtf.models.MnistCNN()
        elif args.model == "mnist_mlp":
            model = dtf.models.MnistMLP(args.hidden_units)
        elif args.model.startswith("resnet"):
            model = getattr(dtf.models, args.model)()
        else:
            from .models import bert
            model = getattr(bert, args.model)()
        model.train()
        opt = _make_optimizer(opt_name, lr, args.model, batch * nrep)
        if args.sync_replicas and server is not None:
            nw = len(server.worker_ranks())
            opt = dtf.train.SyncReplicasOptimizer(
                opt, replicas_to_aggregate=args.replicas_to_aggregate or nw, total_num_replicas=nw)
        global_step = get_or_create_global_step()
        opt.build(list(model.parameters()))

    def train_op():
        if args.model.startswith("bert"):
            b = next(data)
            w = torch.ones_like(b["masked_lm_ids"], dtype=torch.float32)
            loss = model(b["input_ids"], b["segment_ids"], b["input_mask"],
                         b["masked_lm_positions"], b["masked_lm_ids"], w)
        else:
            x, y = next(data)
            logits = model(x)
            if args.model == "mnist_mlp":
                onehot = torch.nn.functional.one_hot(y, 10).to(logits.dtype)
                loss = ops.softmax_cross_entropy_clipped_sum(logits, onehot)
            else:
                loss = ops.sparse_softmax_cross_entropy(logits, y)
        opt.minimize(loss, global_step=global_step)
        return {"loss": loss}

    hooks = [StopAtStepHook(last_step=args.max_steps)]
    cfg = ConfigProto(allow_soft_placement=True, intra_op_parallelism_threads=os.cpu_count(),
                      inter_op_parallelism_threads=os.cpu_count())
    logs = None
    t0, first_step, last = time.time(), None, None
    with MonitoredTrainingSession(master=server.target if server else "", is_chief=is_chief,
                                  checkpoint_dir=args.checkpoint_dir, config=cfg, hooks=hooks,
                                  model=model, optimizer=opt, global_step=global_step,
                                  strategy=strategy, save_checkpoint_steps=args.save_checkpoint_steps,
                                  save_checkpoint_secs=args.save_checkpoint_secs,
                                  log_step_count_steps=None, save_summaries_steps=None) as sess:
        if is_chief and args.log_dir:
            stamp = datetime.datetime.now().strftime("%Y_%m_%d__%H_%M_%S")
            log_directory = os.path.join(args.log_dir, stamp)
            logs = logger.TensorBoardOutputFormat(dir=log_directory)
            print("Logging to", log_directory, flush=True)
        first_step = global_step.value()
        while not sess.should_stop():
            out = sess.run([train_op, "loss", global_step])
            if out is None:
                break
            _, loss, gstep = out
            last = (loss, gstep)
            if is_chief and args.log_every and gstep % args.log_every == 0:
                print("Worker ({}): loss = {:0.2f} (global step: {})".format(
                    args.task_index if server else rid, loss, gstep), flush=True)
                if logs is not None:
                    logs.writekvs({"Global Step": gstep, "Loss": loss}, global_step=gstep)
    if device.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.time() - t0
    if logs is not None:
        logs.close()
    result = {"model": args.model, "strategy": type(strategy).__name__, "replicas": nrep,
              "global_step": global_step.value(), "elapsed_s": round(elapsed, 2),
              "final_loss": None if last is None else round(float(last[0]), 4)}
    steps_done = global_step.value() - (first_step or 0)
    if steps_done > 0 and server is None:
        result["examples_per_sec"] = round(steps_done * batch * nrep / elapsed, 1)
    if args.eval and args.model.startswith("mnist") and is_chief:
        result["test_accuracy"] = evaluate_mnist(model, args, device, dtype)
    if is_chief:
        print(json.dumps(result), flush=True)
    if server is not None:
        server.shutdown()
    return 0


def evaluate_mnist(model, args, device, dtype):
    import torch

    from .data import mnist
    imgs, labels = mnist.load_arrays(args.data_dir, "test")
    model.eval()
    correct = 0
    with torch.no_grad():
        for i in range(0, len(labels), 1000):
            x = torch.as_tensor(imgs[i:i + 1000]).to(device).to(dtype) / 255.0
            pred = model(x).argmax(-1).cpu().numpy()
            correct += int((pred == labels[i:i + 1000]).sum())
    model.train()
    return round(correct / len(labels), 4)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args, _unparsed = build_parser().parse_known_args(argv)
    if (args.num_gpus or 0) > 1 and "WORLD_SIZE" not in os.environ and not args.job_name:
        return _spawn_local(args, argv)
    return run(args)


if __name__ == "__main__":
    sys.exit(main())
