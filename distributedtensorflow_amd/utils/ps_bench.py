"""ResNet-50 under the reference's OWN mode: between-graph, asynchronous parameter server.

``bench.py --strategy ps_async --num-workers W`` (BASELINE.json config 4, "1 PS + N workers",
in the reference's async mode -- ``/root/reference/run_mnist_distributed.py:107-116,142-161``:
workers read the PS variables, compute gradients on their own batch and push them; the PS
applies each push on arrival, Hogwild).  The bench process is the launcher
(``cluster/launcher.py``): it starts 1 PS task + W worker tasks of this same entry point on this
node (workers spread over the node's GPUs, several per GPU when W exceeds them), each task one
process.  The PS keeps the 25.6 M-parameter shard in HBM and exports it with hipIpc; a worker's
push is one device copy into its mailbox slot + a futex post, the owner applies momentum-SGD on
the worker's own HIP stream and answers when that apply's event completes; the pull is one
device copy back (parallel/ps_device.py).

Each worker runs ``warmup`` untimed steps, meets the others at a barrier, times ``steps`` steps
(host clock around device-synchronised boundaries) and writes its record; the launcher reports
images/sec = (W * steps * batch) / max over workers of the timed span, with the per-step push /
wait / pull host times and the PS's apply statistics.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch


def run_task(args):
    """One task of the cluster (``--job_name``/``--task_index`` given by the launcher)."""
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.cluster import ClusterSpec, Config, Server
    from distributedtensorflow_amd.models import resnet50
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import ParameterServerStrategy

    config = Config(args.config)
    ps_hosts, worker_hosts = config.get_ps_and_worker_hosts()
    cluster = ClusterSpec({"ps": list(ps_hosts), "worker": list(worker_hosts)})
    cuda = torch.cuda.is_available()
    ndev = max(torch.cuda.device_count(), 1) if cuda else 1

    def sync():
        if cuda:
            torch.cuda.synchronize()

    if args.job_name == "ps":
        # the PS task is colocated with worker 0 on GPU 0 (device_plan)
        dev = torch.device("cuda", 0) if cuda else torch.device("cpu")
        if cuda:
            torch.cuda.set_device(dev)
        server = Server(cluster, "ps", args.task_index, ps_device=str(dev))
        stats = server.join()
        with open(os.path.join(args.out_dir, f"ps{args.task_index}.json"), "w") as f:
            json.dump({k: v for k, v in stats.items() if isinstance(v, (int, float, str))}, f)
        server.shutdown()
        return
    if cuda:
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", args.task_index)) % ndev)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")       # the flow on CPU (tests); the measured run is on GPUs
    server = Server(cluster, "worker", args.task_index)
    strategy = ParameterServerStrategy(server=server, sync=False, device=dev)
    torch.manual_seed(1234)
    with strategy.scope():
        model = resnet50()
        model.train()
        opt = MomentumOptimizer(args.lr * args.batch / 256, momentum=0.9, weight_decay=1e-4)
        opt.build(list(model.parameters()))
    strategy.register_with_ps(opt, 0)
    client = strategy.ps_client
    g = torch.Generator(device=dev).manual_seed(1234 + args.task_index)
    S = args.image_size
    images = torch.randn(args.batch, S, S, 3, device=dev, generator=g).to(
        torch.bfloat16 if cuda else torch.float32)
    labels = torch.randint(0, 1000, (args.batch,), device=dev, generator=g)

    def step():
        loss = ops.sparse_softmax_cross_entropy(model(images), labels)
        opt.minimize(loss)
        return loss

    reducer = opt._reducer
    timings = dict(client.timing)
    timings.update(getattr(reducer, "timing", {}))
    for _ in range(args.warmup):
        loss = step()
    opt.synchronize_variables()          # the pipelined push in flight completes
    sync()
    for v in timings.values():
        v.clear()
    import torch.distributed as dist
    dist.barrier(group=server.worker_group)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    opt.synchronize_variables()          # inside the timed region: the last push is answered
    sync()
    elapsed = time.perf_counter() - t0
    rec = {"worker": args.task_index, "elapsed_s": elapsed, "steps": args.steps,
           "batch": args.batch, "loss": float(loss), "device": str(dev),
           "global_step": client.global_step, "data_plane": client.data_plane_in_use,
           "pipelined": bool(getattr(reducer, "_pipe", False)),
           **{f"{k}_per_step": round(sum(v) / max(len(v), 1), 3) for k, v in timings.items()}}
    with open(os.path.join(args.out_dir, f"worker{args.task_index}.json"), "w") as f:
        json.dump(rec, f)
    client.stop()
    dist.barrier(group=server.worker_group)
    server.shutdown()


def device_plan(num_workers, gpus, visible):
    """(worker device indices, PS device index) of ``bench.py --strategy ps_async --gpus N``:
    worker i on GPU ``i % N`` (one per GPU when W = N, round-robin when W > N), the PS task
    colocated on GPU 0 (BASELINE config 4, "1 PS + N workers colocated on one node").  Refuses
    (ValueError) to plan for more GPUs than are visible: a run labelled N GPUs must use N.
    ``visible`` = 0 (a CPU-only host) plans a CPU run for N = 1: no devices."""
    if gpus < 1 or num_workers < 1:
        raise ValueError("ps_async needs --gpus >= 1 and --num-workers >= 1")
    if visible == 0 and gpus == 1:
        return [None] * num_workers, None
    if visible < gpus:
        raise ValueError(f"--gpus {gpus} but only {visible} GPU(s) are visible: refusing to "
                         f"measure fewer GPUs than requested")
    return [i % gpus for i in range(num_workers)], 0


def run_launcher(args, metric_note=""):
    """Start 1 PS + W workers of ``bench.py`` on this node and report the aggregate."""
    import tempfile

    from distributedtensorflow_amd.cluster.launcher import launch_local
    from distributedtensorflow_amd.utils import dtf_env
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    # device_count() does not initialise the GPU (the tasks are fresh processes anyway)
    visible = torch.cuda.device_count()
    try:
        workers_dev, ps_dev = device_plan(args.num_workers, args.gpus, visible)
    except ValueError as e:
        print(f"bench.py: error: {e}", file=sys.stderr, flush=True)
        raise SystemExit(2)
    work = tempfile.mkdtemp(prefix="dtf_ps_bench_")
    extra = ["--strategy", "ps_async", "--batch", str(args.batch), "--steps", str(args.steps),
             "--warmup", str(args.warmup), "--image-size", str(args.image_size),
             "--lr", str(args.lr), "--out-dir", work, "--gpus", str(args.gpus)]
    # worker i -> LOCAL_RANK i % N (launch_local); CPU-only hosts (tests): the PS keeps its shard
    # in host memory (/dev/shm plane)
    codes, logs = launch_local(os.path.join(root, "bench.py"), 1, args.num_workers, work, extra,
                               env={"PYTHONPATH": root}, timeout_s=args.timeout,
                               gpus_per_host=args.gpus if ps_dev is not None else None)
    if any(c != 0 for c in codes.values()):
        for k, p in logs.items():
            sys.stderr.write(f"--- {k}\n" + open(p).read()[-3000:])
        raise SystemExit(f"ps_async bench failed: {codes}")
    recs = [json.load(open(os.path.join(work, f"worker{i}.json")))
            for i in range(args.num_workers)]
    ps = json.load(open(os.path.join(work, "ps0.json")))
    span = max(r["elapsed_s"] for r in recs)
    imgs = sum(r["steps"] * r["batch"] for r in recs)
    ips = imgs / span
    per = {k: round(sum(r.get(k, 0.0) for r in recs) / len(recs), 3)
           for k in ("copy_sync_ms_per_step", "wait_ms_per_step", "pull_ms_per_step",
                     "fence_ms_per_step", "answer_ms_per_step")}
    applied = max(int(ps.get("applied", 0)), 1)
    used = sorted({r["device"] for r in recs if r["device"].startswith("cuda")})
    if ps_dev is not None and used != [f"cuda:{i}" for i in sorted(set(workers_dev))]:
        raise SystemExit(f"ps_async bench: workers ran on {used}, planned {sorted(set(workers_dev))}")
    rec = {"metric": "images/sec ResNet-50 async parameter server (between-graph, 1 PS + "
                     f"{args.num_workers} workers)",
           "value": round(ips, 2), "unit": "images/sec", "n_gpus": len(used),
           "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(span / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (random NHWC 224x224x3 images, random labels; random-init weights)",
           "config": {"model": "resnet50", "global_batch": args.batch * args.num_workers,
                      "per_gpu_batch": args.batch, "image_size": args.image_size,
                      "parallelism": f"ps1+async{args.num_workers}",
                      "optimizer": "momentum0.9+wd1e-4 applied on the PS (Hogwild)",
                      "data_plane": recs[0]["data_plane"],
                      "pipelined_push_pull": all(r.get("pipelined") for r in recs),
                      "worker_devices": [r["device"] for r in recs],
                      "ps_device": None if ps_dev is None else f"cuda:{ps_dev}",
                      "worker_host_ms_per_step": per,
                      "ps_apply_ms_mean": round(1e3 * float(ps.get("apply_s", 0.0)) / applied, 3),
                      "ps_applied": ps.get("applied"), "ps_pushes": ps.get("pushes"),
                      "ps_max_inflight_applies": ps.get("max_inflight"),
                      "final_global_step": max(r["global_step"] for r in recs),
                      "final_loss": [round(r["loss"], 4) for r in recs], "note": metric_note,
                      "dtf_env": dtf_env()}}
    print(json.dumps(rec), flush=True)
    return rec
