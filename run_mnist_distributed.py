#!/usr/bin/env python
"""Drop-in equivalent of the reference's ``run_mnist_distributed.py`` on distributedtensorflow_amd.

    python run_mnist_distributed.py --job_name=ps     --task_index=0
    python run_mnist_distributed.py --job_name=worker --task_index=0   # chief
    python run_mnist_distributed.py --job_name=worker --task_index=1

Same behaviour as the reference (``run_mnist_distributed.py:73-182``): cluster from
``config.json`` (``{"ps": {...}, "workers": {...}}``, task order = JSON order), one process per
task, PS tasks host the variables and block in ``server.join()`` (here: returning cleanly when
the workers are done or on Ctrl+C), workers train the reference CNN with Adam(5e-4) on batches of
128 asynchronously (between-graph PS) until ``global_step`` reaches 1000, and the chief prints
``Worker (i): loss = x.xx (global step: n)`` and writes ``Global Step`` / ``Loss`` TensorBoard
scalars to ``/tmp/distributed_logs/<timestamp>``.  Extra flags: ``--sync_replicas``,
``--max_steps``, ``--config``, ``--data_dir``, ``--log_dir``, ``--checkpoint_dir``.
Workers use their GPU (``LOCAL_RANK``/task-index) when present, the CPU otherwise.
"""
from __future__ import annotations

import argparse
import datetime
import faulthandler
import os
import signal
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FLAGS = None


def main():
    import torch

    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.cluster import ClusterSpec, Config, Server
    from distributedtensorflow_amd.data import mnist
    from distributedtensorflow_amd.models import MnistCNN
    from distributedtensorflow_amd.parallel import ParameterServerStrategy
    from distributedtensorflow_amd.summary import logger
    from distributedtensorflow_amd.train import (ConfigProto, MonitoredTrainingSession,
                                                 StopAtStepHook, get_or_create_global_step)

    if FLAGS.seed is not None:           # default: unseeded random init, like the reference
        torch.manual_seed(FLAGS.seed)

    print("run main with args =", FLAGS, flush=True)
    config = Config(FLAGS.config)
    ps_hosts, worker_hosts = config.get_ps_and_worker_hosts()
    cluster = ClusterSpec({"ps": list(ps_hosts), "worker": list(worker_hosts)})
    ps_device = FLAGS.ps_device
    if ps_device == "auto":
        ps_device = "gpu" if torch.cuda.is_available() else "cpu"
    ps_device = (f"cuda:{FLAGS.task_index % torch.cuda.device_count()}" if ps_device == "gpu"
                 else "cpu")
    server = Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_index,
                    ps_device=ps_device)

    if FLAGS.job_name == "ps":
        if ps_device != "cpu":
            torch.cuda.set_device(torch.device(ps_device))
        print("Started Parameter Server ...", flush=True)
        stats = server.join()
        Server.exit_for_rejoin(stats)       # a peer died: restart in the cluster's new epoch
        print("Close Parameter Server ...", stats, flush=True)
        if not stats.get("interrupted"):
            server.shutdown()
        return
    if FLAGS.job_name != "worker":
        raise ValueError("--job_name must be 'ps' or 'worker'")

    is_chief = FLAGS.task_index == 0
    if FLAGS.device == "auto":
        use_gpu = torch.cuda.is_available()
    else:
        use_gpu = FLAGS.device == "gpu"
    if use_gpu:
        ndev = torch.cuda.device_count()
        device = torch.device("cuda", FLAGS.task_index % ndev)   # task_index % num_gpus (R7)
    else:
        device = torch.device("cpu")
    if FLAGS.dtype == "auto":
        dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    else:   # fp32 = the reference's own precision (dataset.py:93-95, tf.layers default dtype)
        dtype = torch.bfloat16 if FLAGS.dtype == "bf16" else torch.float32

    # input pipeline: ds.repeat().batch(128).prefetch(...) (reference :77-85) -- same order, no
    # shuffle, every worker the same batches; on a GPU the whole uint8 set lives in HBM and each
    # batch is one fused gather + u8->float/255 kernel (data/device.py), no per-step H2D copy
    batch_size = FLAGS.batch_size
    imgs, labels = mnist.load_arrays(FLAGS.data_dir, "train")
    if device.type == "cuda":
        it = dtf.data.DeviceArrayDataset(imgs, labels, batch_size, device, dtype=dtype)
    else:
        ds = (dtf.data.Dataset.from_tensor_slices((imgs, labels))
              .repeat().batch(batch_size).prefetch(4))
        it = iter(ds)

    strategy = ParameterServerStrategy(server=server, sync=FLAGS.sync_replicas, device=device,
                                       data_plane=FLAGS.data_plane)
    with strategy.scope():
        model = MnistCNN()
        opt = dtf.train.AdamOptimizer(FLAGS.learning_rate)
        if dtype == torch.float32:
            opt.shadow_dtype = None          # fp32 compute reads the fp32 masters directly
        if FLAGS.sync_replicas:
            opt = dtf.train.SyncReplicasOptimizer(opt, replicas_to_aggregate=len(worker_hosts),
                                                  total_num_replicas=len(worker_hosts))
        global_step = get_or_create_global_step()
        opt.build(list(model.parameters()))

    def train_op():
        x, y = next(it)
        if device.type != "cuda":
            x = torch.as_tensor(x).to(dtype) / 255.0
            y = torch.as_tensor(y).long()
        loss = ops.sparse_softmax_cross_entropy(model(x), y)
        opt.minimize(loss, global_step=global_step)
        return {"loss": loss}

    hooks = [StopAtStepHook(last_step=FLAGS.max_steps)]
    tf_config = ConfigProto(allow_soft_placement=True,
                            intra_op_parallelism_threads=os.cpu_count(),
                            inter_op_parallelism_threads=os.cpu_count())
    import time
    t_start, first_step = None, None
    with MonitoredTrainingSession(master=server.target, is_chief=is_chief,
                                  checkpoint_dir=FLAGS.checkpoint_dir, config=tf_config,
                                  hooks=hooks, model=model, optimizer=opt,
                                  global_step=global_step, strategy=strategy,
                                  save_checkpoint_steps=FLAGS.save_checkpoint_steps,
                                  log_step_count_steps=None, save_summaries_steps=None) as mon_sess:
        if is_chief:
            date_string = datetime.datetime.now().strftime("%Y_%m_%d__%H_%M_%S")
            log_directory = os.path.join(FLAGS.log_dir, date_string)
            logs = logger.TensorBoardOutputFormat(dir=log_directory)
            print("Logging to", log_directory, flush=True)
        while not mon_sess.should_stop():
            if t_start is None:
                t_start = time.time()
            if is_chief:
                out = mon_sess.run([train_op, "loss", global_step])
                if out is None:
                    break
                _, train_loss, gstep = out
                print("Worker ({}): loss = {:0.2f} (global step: {})".format(
                    FLAGS.task_index, train_loss, gstep), flush=True)
                logs.writekvs({"Global Step": gstep, "Loss": train_loss}, global_step=gstep)
            else:
                mon_sess.run(train_op)
    if mon_sess.recoveries:
        print(f"Recovered {mon_sess.recoveries} time(s) from a failed task", flush=True)
    if is_chief:
        logs.close()
        if t_start is not None:
            # reference template prints the same (templates/00_mnist_replica.py:265)
            print("Training elapsed time: %.2f s" % (time.time() - t_start), flush=True)
    server.shutdown()


def parse(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--job_name", type=str, default="", required=True,
                        help="One of 'ps', 'worker'")
    parser.add_argument("--task_index", type=int, required=True,
                        help="Index of task within the job")
    parser.add_argument("--config", default="config.json")
    parser.add_argument("--max_steps", type=int, default=1000)
    parser.add_argument("--batch_size", type=int, default=128)
    parser.add_argument("--learning_rate", type=float, default=0.0005)
    parser.add_argument("--data_dir", default="/tmp/data/")
    parser.add_argument("--log_dir", default="/tmp/distributed_logs")
    parser.add_argument("--checkpoint_dir", default=None)
    parser.add_argument("--save_checkpoint_steps", type=int, default=None,
                        help="chief checkpoints every N global steps (default: every 600 s)")
    parser.add_argument("--sync_replicas", action="store_true")
    parser.add_argument("--seed", type=int, default=None,
                        help="seed the variable initialisers (reproducible runs; not a reference "
                             "flag)")
    parser.add_argument("--device", choices=("auto", "cpu", "gpu"), default="auto")
    parser.add_argument("--dtype", choices=("auto", "bf16", "fp32"), default="fp32",
                        help="compute dtype: fp32 (default) = the reference's precision "
                             "(dataset.py:93-95, tf.layers' float32; f32 MFMA kernels on GPUs); "
                             "bf16 = opt-in bf16 compute with fp32 masters; auto = bf16 on GPUs, "
                             "fp32 on CPUs")
    parser.add_argument("--ps_device", choices=("auto", "cpu", "gpu"), default="auto",
                        help="where a ps task keeps its variable shard (auto: its GPU's HBM)")
    parser.add_argument("--data_plane", choices=("auto", "ipc", "shm", "gloo"), default=None,
                        help="PS push/pull transport: auto = HBM shard mapped over hipIpc (GPU "
                             "PS) or /dev/shm (CPU PS); gloo = host tensors over TCP "
                             "(cross-host clusters)")
    flags, _unparsed = parser.parse_known_args(argv)
    return flags


if __name__ == "__main__":
    # `kill -USR1 <pid>` (the launcher does it before tearing down a timed-out job) writes every
    # thread's Python stack into this task's log
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    FLAGS = parse()
    main()
