#!/usr/bin/env python
"""All-reduce bus-bandwidth sweep (explain the 1->8 GPU curve before running it).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/allreduce_bw.py [--min-mb 1 --max-mb 256 --dtype fp32 --iters 20]

One process per GPU over RCCL (xGMI); ``--backend gloo`` runs the same sweep on CPU.  For each
message size S it times ``iters`` back-to-back ``all_reduce`` calls between barriers and reports

    algbw = S / t,      busbw = algbw * 2 (N - 1) / N

(busbw is the per-link rate a ring moves; on MI355X each GPU has 7 xGMI links of ~153 GB/s, so a
single ring tops out near one link's rate).  It also reports the bucketed-gradient case the
trainer actually issues: ResNet-50's 102 MB of fp32 gradients cut into the strategy's buckets,
launched back to back (what MirroredStrategy overlaps with backward).  Rank 0 prints one JSON
line per size and a summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-mb", type=float, default=1)
    ap.add_argument("--max-mb", type=float, default=256)
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default=None)
    ap.add_argument("--bucket-mb", type=float, default=64)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from distributedtensorflow_amd.parallel import init_process_group_from_env
    backend = a.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    init_process_group_from_env(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else \
        torch.device("cpu")
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    esz = torch.tensor([], dtype=dt).element_size()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dist.barrier()

    def timed(fn, iters):
        for _ in range(a.warmup):
            fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        sync()
        t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64)
        if backend == "nccl":
            t = t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    rows = []
    mb = a.min_mb
    while mb <= a.max_mb + 1e-9:
        n = max(1, int(mb * 2**20) // esz)
        x = torch.ones(n, dtype=dt, device=dev)
        t = timed(lambda: dist.all_reduce(x), a.iters)
        alg = n * esz / t / 1e9
        row = {"size_mb": round(n * esz / 2**20, 3), "time_us": round(t * 1e6, 1),
               "algbw_GBps": round(alg, 2), "busbw_GBps": round(alg * 2 * (world - 1) / world, 2)}
        rows.append(row)
        if rank == 0:
            print(json.dumps({"n": world, "backend": backend, "dtype": a.dtype, **row}),
                  flush=True)
        mb *= 2
    # the trainer's pattern: ResNet-50 fp32 gradients (25.56 M params) in buckets, async
    total = 25_557_032
    bucket = max(1, int(a.bucket_mb * 2**20) // 4)
    g = torch.ones(total, dtype=torch.float32, device=dev)

    def bucketed():
        works = [dist.all_reduce(g[s:s + bucket], async_op=True) for s in range(0, total, bucket)]
        for w in works:
            w.wait()
    t = timed(bucketed, max(3, a.iters // 4))
    summary = {"n": world, "backend": backend, "resnet50_fp32_grad_mb": round(total * 4 / 2**20, 1),
               "bucket_mb": a.bucket_mb, "bucketed_allreduce_ms": round(t * 1e3, 3),
               "bucketed_busbw_GBps": round(total * 4 / t / 1e9 * 2 * (world - 1) / world, 2),
               "peak_busbw_GBps": max(r["busbw_GBps"] for r in rows)}
    if rank == 0:
        print(json.dumps(summary), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                for r in rows:
                    f.write(json.dumps({"n": world, "backend": backend, "dtype": a.dtype, **r})
                            + "\n")
                f.write(json.dumps(summary) + "\n")
    dist.barrier()
    dist.destroy_process_group()
    return rows, summary


if __name__ == "__main__":
    main()
