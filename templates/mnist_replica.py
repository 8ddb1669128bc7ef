#!/usr/bin/env python
"""Distributed MNIST MLP with optional synchronous replicas (reference
``templates/00_mnist_replica.py``): Supervisor-managed
session, SyncReplicasOptimizer(Adam) aggregation with stale-gradient drop, per-worker GPU
assignment (``task_index % num_gpus``), ``--existing_servers`` (attach to a rendezvous that was
already set up: RANK/WORLD_SIZE/MASTER_* in the environment), feed-style ``next_batch`` training,
elapsed time and validation cross-entropy at the end.

    python templates/mnist_replica.py --job_name=ps --task_index=0
    python templates/mnist_replica.py --job_name=worker --task_index=0 --sync_replicas
    python templates/mnist_replica.py --job_name=worker --task_index=1 --sync_replicas
"""
import argparse
import math
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FLAGS = None
IMAGE_PIXELS = 28


def main():
    import torch

    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.cluster import ClusterSpec, Server
    from distributedtensorflow_amd.data import mnist
    from distributedtensorflow_amd.parallel import ParameterServerStrategy

    data = mnist.read_data_sets(FLAGS.data_dir, one_hot=True)
    if FLAGS.download_only:
        sys.exit(0)
    if FLAGS.job_name not in ("ps", "worker"):
        raise ValueError("Must specify an explicit `job_name`")
    print("job name = %s" % FLAGS.job_name)
    print("task index = %d" % FLAGS.task_index)

    cluster = ClusterSpec({"ps": FLAGS.ps_hosts.split(","),
                           "worker": FLAGS.worker_hosts.split(",")})
    num_workers = cluster.num_tasks("worker")
    if FLAGS.existing_servers:
        # the rendezvous was created outside this script (e.g. by torchrun / a cluster manager)
        from distributedtensorflow_amd.parallel import init_process_group_from_env
        init_process_group_from_env("gloo")
        server = Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_index)
    else:
        server = Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_index)
    if FLAGS.job_name == "ps":
        stats = server.join()
        server.exit_for_rejoin(stats)      # a peer died and was restarted: new cluster epoch
        if not stats.get("interrupted"):
            server.shutdown()
        return

    is_chief = FLAGS.task_index == 0
    if FLAGS.num_gpus > 0 and torch.cuda.is_available():
        device = torch.device("cuda", FLAGS.task_index % FLAGS.num_gpus)   # R7
    else:
        device = torch.device("cpu")
    strategy = ParameterServerStrategy(server=server, sync=FLAGS.sync_replicas, device=device)
    with strategy.scope():
        global_step = dtf.train.get_or_create_global_step()
        model = dtf.models.MnistMLP(FLAGS.hidden_units)
        opt = dtf.train.AdamOptimizer(FLAGS.learning_rate)
        opt.shadow_dtype = None      # fp32 end to end, like the reference's MLP
        if FLAGS.sync_replicas:
            replicas = FLAGS.replicas_to_aggregate or num_workers
            opt = dtf.train.SyncReplicasOptimizer(opt, replicas_to_aggregate=replicas,
                                                  total_num_replicas=num_workers,
                                                  name="mnist_sync_replicas")
        opt.build(list(model.parameters()))

    def cross_entropy(x, y):
        return ops.softmax_cross_entropy_clipped_sum(model(x), y)

    sv = dtf.train.Supervisor(is_chief=is_chief, logdir=tempfile.mkdtemp(),
                              recovery_wait_secs=1, global_step=global_step, model=model,
                              optimizer=opt, strategy=strategy)
    sess_config = dtf.train.ConfigProto(allow_soft_placement=True, log_device_placement=False,
                                        device_filters=["/job:ps",
                                                        "/job:worker/task:%d" % FLAGS.task_index])
    if is_chief:
        print("Worker %d: Initializing session..." % FLAGS.task_index)
    else:
        print("Worker %d: Waiting for session to be initialized..." % FLAGS.task_index)
    sess = sv.prepare_or_wait_for_session(server.target, config=sess_config)
    print("Worker %d: Session initialization complete." % FLAGS.task_index)

    time_begin = time.time()
    print("Training begins @ %f" % time_begin)
    local_step = 0
    while True:
        xs, ys = data.train.next_batch(FLAGS.batch_size)

        def train_step():
            loss = cross_entropy(torch.as_tensor(xs, device=device),
                                 torch.as_tensor(ys, device=device))
            opt.minimize(loss, global_step=global_step)
            return {"loss": loss}
        out = sess.run([train_step, global_step])
        if out is None:
            break
        step = out[1]
        local_step += 1
        now = time.time()
        print("%f: Worker %d: training step %d done (global step: %d)" %
              (now, FLAGS.task_index, local_step, step))
        if step >= FLAGS.train_steps:
            break
    time_end = time.time()
    print("Training ends @ %f" % time_end)
    print("Training elapsed time: %f s" % (time_end - time_begin))
    with torch.no_grad():
        val_xent = float(cross_entropy(torch.as_tensor(data.validation.images, device=device),
                                       torch.as_tensor(data.validation.labels, device=device)))
    print("After %d training step(s), validation cross entropy = %g" %
          (FLAGS.train_steps, val_xent))
    sv.stop()
    server.shutdown()


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--data_dir", default="/tmp/mnist-data")
    p.add_argument("--download_only", action="store_true")
    p.add_argument("--task_index", type=int, default=None)
    p.add_argument("--num_gpus", type=int, default=0)
    p.add_argument("--replicas_to_aggregate", type=int, default=None)
    p.add_argument("--hidden_units", type=int, default=100)
    p.add_argument("--train_steps", type=int, default=200)
    p.add_argument("--batch_size", type=int, default=100)
    p.add_argument("--learning_rate", type=float, default=0.01)
    p.add_argument("--sync_replicas", action="store_true")
    p.add_argument("--existing_servers", action="store_true")
    p.add_argument("--ps_hosts", default="localhost:2222")
    p.add_argument("--worker_hosts", default="localhost:2223,localhost:2224")
    p.add_argument("--job_name", default=None)
    FLAGS, _ = p.parse_known_args()
    if FLAGS.task_index is None or FLAGS.task_index == "":
        raise ValueError("Must specify an explicit `task_index`")
    main()
