"""Eager vs HIP-graph-replayed training steps (train/graphed.py) on launch-bound workloads: the
reference MNIST CNN at the reference batch (128; bf16 and fp32 compute, Adam) and ResNet-50 at
small per-GPU batches.  Prints one JSON line per (workload, mode).

    python tools/graph_step_bench.py [--steps 200] [--out graph_steps.jsonl]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(workload, dtype):
    import distributedtensorflow_amd as dtf
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import MnistCNN, resnet50
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import OneDeviceStrategy
    torch.manual_seed(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    with OneDeviceStrategy("/gpu:0").scope():
        if workload == "mnist_cnn":
            model = MnistCNN()
            opt = dtf.train.AdamOptimizer(5e-4)      # run_mnist_distributed.py:116
            if dtype == torch.float32:
                opt.shadow_dtype = None
            x = torch.rand(128, 784, device="cuda", generator=g).to(dtype)
            y = torch.randint(0, 10, (128,), device="cuda", generator=g)
        else:
            b = int(workload.split("_b")[1])
            model = resnet50()
            opt = MomentumOptimizer(0.1, 0.9, weight_decay=1e-4)
            x = torch.randn(b, 224, 224, 3, device="cuda", generator=g).bfloat16()
            y = torch.randint(0, 1000, (b,), device="cuda", generator=g)
        opt.build(list(model.parameters()))

    def step(xx, yy):
        loss = ops.sparse_softmax_cross_entropy(model(xx), yy)
        opt.minimize(loss)
        return loss
    return step, opt, x, y


def timed(fn, steps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--out", default=None)
    ap.add_argument("--workloads", default="mnist_cnn:bf16,mnist_cnn:fp32,resnet50_b16:bf16,"
                                          "resnet50_b64:bf16")
    a = ap.parse_args()
    from distributedtensorflow_amd.train import GraphedTrainStep
    rows = []
    for wl in a.workloads.split(","):
        name, dt = wl.split(":")
        dtype = torch.bfloat16 if dt == "bf16" else torch.float32
        step, opt, x, y = build(name, dtype)
        steps = a.steps if name == "mnist_cnn" else max(20, a.steps // 10)
        eager = timed(lambda: step(x, y), steps)
        g = GraphedTrainStep(step, opt, [x, y], warmup=2)
        graphed = timed(lambda: g(x, y), steps)
        for mode, ms in (("eager", eager), ("hip_graph", graphed)):
            row = {"workload": name, "dtype": dt, "mode": mode, "ms_per_step": round(ms, 4),
                   "steps": steps}
            if mode == "hip_graph":
                row["speedup_vs_eager"] = round(eager / ms, 2)
            rows.append(row)
            print(json.dumps(row), flush=True)
        del g, step, opt, x, y
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
