#!/usr/bin/env python
"""Between-graph replication, asynchronous parameter server (reference
``templates/00_between_graph_replication_async_mnist.py``), made runnable: the reference skeleton
leaves ``loss = ...``; here it is the MNIST MLP.  Adagrad(0.01), StopAtStepHook, and a
MonitoredTrainingSession with ``checkpoint_dir`` (chief restores / saves TF-V2 checkpoints).

    python templates/between_graph_async_mnist.py --job_name=ps --task_index=0 \
        --ps_hosts=127.0.0.1:2222 --worker_hosts=127.0.0.1:2223,127.0.0.1:2224
    python templates/between_graph_async_mnist.py --job_name=worker --task_index=0 ...
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FLAGS = None


def main():
    import torch

    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.cluster import ClusterSpec, Server
    from distributedtensorflow_amd.data import DeviceArrayDataset, mnist
    from distributedtensorflow_amd.parallel import ParameterServerStrategy

    cluster = ClusterSpec({"ps": FLAGS.ps_hosts.split(","),
                           "worker": FLAGS.worker_hosts.split(",")})
    server = Server(cluster, job_name=FLAGS.job_name, task_index=FLAGS.task_index)
    if FLAGS.job_name == "ps":
        stats = server.join()
        server.exit_for_rejoin(stats)      # a peer died and was restarted: new cluster epoch
        if not stats.get("interrupted"):
            server.shutdown()
        return
    device = torch.device("cpu")
    strategy = ParameterServerStrategy(server=server, device=device)
    imgs, labels = mnist.load_arrays(FLAGS.data_dir, "train")
    data = DeviceArrayDataset(imgs, labels, FLAGS.batch_size, device)
    with strategy.scope():
        model = dtf.models.MnistMLP(FLAGS.hidden_units)
        global_step = dtf.train.get_or_create_global_step()
        opt = dtf.train.AdagradOptimizer(0.01)
        opt.build(list(model.parameters()))

    def train_op():
        x, y = next(data)
        loss = ops.sparse_softmax_cross_entropy(model(x), y)
        opt.minimize(loss, global_step=global_step)
        return {"loss": loss}

    hooks = [dtf.train.StopAtStepHook(last_step=FLAGS.train_steps)]
    with dtf.train.MonitoredTrainingSession(master=server.target,
                                            is_chief=(FLAGS.task_index == 0),
                                            checkpoint_dir=FLAGS.checkpoint_dir,
                                            hooks=hooks, model=model, optimizer=opt,
                                            global_step=global_step,
                                            strategy=strategy) as mon_sess:
        while not mon_sess.should_stop():
            mon_sess.run(train_op)     # asynchronous step; recovers from a lost PS peer
    print(f"worker {FLAGS.task_index} done at global step {global_step.value()}", flush=True)
    server.shutdown()


if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("--ps_hosts", default="127.0.0.1:2222")
    parser.add_argument("--worker_hosts", default="127.0.0.1:2223,127.0.0.1:2224")
    parser.add_argument("--job_name", default="", help="One of 'ps', 'worker'")
    parser.add_argument("--task_index", type=int, default=0)
    parser.add_argument("--train_steps", type=int, default=1000000)
    parser.add_argument("--batch_size", type=int, default=100)
    parser.add_argument("--hidden_units", type=int, default=100)
    parser.add_argument("--data_dir", default="/tmp/mnist-data")
    parser.add_argument("--checkpoint_dir", default="/tmp/train_logs")
    FLAGS, _ = parser.parse_known_args()
    main()
