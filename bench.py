#!/usr/bin/env python
"""North-star benchmark: ResNet-50 training images/sec on MI355X (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W [--batch 256] [--impl dtf|torch]

For N > 1 the bench runs one process per GPU (RCCL over xGMI), either under
``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` or launched by
bench.py itself: without torchrun's ``WORLD_SIZE`` in the environment, ``--gpus N`` spawns the N
rank processes BEFORE any GPU call, relays their output (rank 0 prints the JSON line) and exits
with the worst rank's exit code.  It never measures fewer GPUs than asked: fewer visible devices
than N, or a ``WORLD_SIZE`` that differs from N, is a non-zero exit with the reason.

Each rank trains on its own synthetic ImageNet-shaped batch (weak scaling: per-GPU batch fixed);
the timed region is exactly K full training steps (forward, backward, overlapped bucketed
all-reduce, fused SGD-momentum update) bracketed by a barrier + device synchronize on both sides;
the MAX elapsed time over ranks is reported.

Hangs end loudly: the process group and the collective watchdog (parallel/watchdog.py) use
``DTF_COMM_TIMEOUT_S`` (default 300 s), and a stack-dumping deadline (``faulthandler``) bounds
the warm-up (``--warmup-timeout``) and every timed step (``--step-timeout``): on expiry every
thread's stack goes to stderr and the process exits non-zero.

``--impl dtf``   (default) this framework: hand-written HIP kernels, MirroredStrategy.
``--impl torch`` the stock PyTorch-ROCm comparator (MIOpen convs, DDP) on the same data.
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import signal
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) ResNet-50 synthetic ImageNet at 1/2/4/8 MI355X"
BASELINE_VALUE = None   # the reference publishes no ResNet-50 number


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=None,
                   help="per-GPU batch (default 1984 for ResNet-50: ~80 GB of the 288 GB HBM3E; "
                        "the conv kernels rebase their buffer descriptors per tile, so no 2 GiB "
                        "tensor cap remains).  1984 = 31 x 64 fills whole rounds of 256-row tiles "
                        "on the 256 CUs in the GEMM-routed stage-3/4 convs (M = B*196 and B*49: "
                        "1984 -> 1519 / 380 tiles per 256-wide N slab, the tile rounds 0.99 "
                        "busy; 2048 -> 1568 / 392, 0.875 / 0.766); same-box sweeps "
                        "1856/1920/1984/2006/2048/2112/2240/2304/2560/3072 -> 1984 best, +1.7-2.3 %% "
                        "over 2048 (profiles/measurements/r2_resnet_batch_sweep_tile_rounds_*.jsonl); "
                        "512 sequences for BERT: sweep 128/256/512/1024 -> 875k/1.03M/1.14M/1.15M "
                        "tok/s)")
    p.add_argument("--impl", choices=("dtf", "torch"), default="dtf")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--bucket-mb", default=None,
                   help="all-reduce bucket size in MB, or 'auto' (the default when N > 1; 64 at "
                        "N = 1, where nothing is reduced): after the warm-up, time 2 steps at each "
                        "of 16/32/64/128 MB (max over ranks) and keep the fastest for the timed "
                        "steps (SURVEY.md 5.8)")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--cudnn-benchmark", type=int, default=1,
                   help="--impl torch: 1 = MIOpen exhaustive algorithm search on first use "
                        "(slow to warm up at large batch), 0 = MIOpen immediate mode (heuristic "
                        "/ find-db solutions, no search)")
    p.add_argument("--dump-master", default=None,
                   help="after the timed steps, save the (rank-0) fp32 master weights to this "
                        "file (tests compare the forced-reducer run bit for bit with the plain one)")
    p.add_argument("--model", choices=("resnet50", "bert_base"), default="resnet50",
                   help="resnet50: the headline metric; bert_base: BASELINE config 5 "
                        "(MLM, LAMB, MultiWorkerMirroredStrategy) in tokens/sec")
    p.add_argument("--strategy", choices=("mirrored", "ps", "ps_async"), default="mirrored",
                   help="mirrored: MirroredStrategy (bucketed RCCL all-reduce overlapped with "
                        "backward); ps: BASELINE config 4, colocated synchronous "
                        "ParameterServerStrategy (--num-ps owner ranks; 1 = '1 PS + N workers', "
                        "= N: sharded owners, reduce-scatter / all-gather); ps_async: config 4 in "
                        "the reference's own mode -- this process launches 1 PS task + "
                        "--num-workers worker tasks (between-graph, Hogwild pushes applied on "
                        "arrival; utils/ps_bench.py)")
    p.add_argument("--num-ps", type=int, default=1)
    p.add_argument("--num-workers", type=int, default=None,
                   help="ps_async: worker tasks (default: --gpus, one worker per GPU; more "
                        "workers than GPUs share them round-robin)")
    p.add_argument("--timeout", type=float, default=900, help="ps_async: launcher timeout (s)")
    # set by the ps_async launcher on its tasks (cluster/launcher.py)
    p.add_argument("--job_name", default=None, help=argparse.SUPPRESS)
    p.add_argument("--task_index", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--config", default=None, help=argparse.SUPPRESS)
    p.add_argument("--out-dir", default=None, help=argparse.SUPPRESS)
    p.add_argument("--seq-len", type=int, default=128)
    p.add_argument("--max-predictions", type=int, default=20)
    p.add_argument("--gemm-tuning", choices=("auto", "off", "tune"), default="auto",
                   help="hipBLASLt solution choice for the library GEMMs (PyTorch TunableOp): "
                        "auto = use this repo's tuned table for the model when present, tune = "
                        "benchmark every solution once and write the table to --gemm-tuning-out")
    p.add_argument("--gemm-tuning-out", default=None)
    p.add_argument("--warmup-timeout", type=float, default=900,
                   help="seconds the warm-up may take before the bench dumps every thread's "
                        "stack and exits non-zero (0 = no deadline)")
    p.add_argument("--step-timeout", type=float, default=120,
                   help="seconds any timed step (and the final drain) may take before the bench "
                        "dumps stacks and exits non-zero (0 = no deadline)")
    args = p.parse_args()
    if args.bucket_mb is None:
        args.bucket_mb = "auto" if args.gpus > 1 else "64"
    args.bucket_auto = args.bucket_mb == "auto"
    args.bucket_mb = 64.0 if args.bucket_auto else float(args.bucket_mb)
    if args.num_workers is None:
        args.num_workers = max(args.gpus, 1)
    if args.batch is None:
        args.batch = 512 if args.model == "bert_base" else 1984
    return args


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return None


def _rccl_debug_file():
    """N > 1 on RCCL: have the communicator log its INIT lines to a per-rank file (unless the
    user set NCCL_DEBUG), so the JSON can carry the channel count RCCL itself reports."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 or "NCCL_DEBUG" in os.environ or \
            os.environ.get("DTF_BENCH_BACKEND", "nccl") != "nccl":
        return None
    path = f"/tmp/dtf_rccl_init_{os.getpid()}.log"
    os.environ.update({"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT",
                       "NCCL_DEBUG_FILE": path})
    return path


def _rccl_channels(path):
    """Channel count from RCCL's own INIT log: '<n> coll channels' (NCCL >= 2.12 format), else
    the ring count of its 'Channel NN/MM' lines; None when unavailable."""
    import re
    if not path or not os.path.exists(path):
        return None
    text = open(path, errors="replace").read()
    m = re.findall(r"(\d+) coll channels", text)
    if m:
        return int(m[-1])
    m = re.findall(r"Channel \d+/(\d+)", text)
    return int(m[-1]) if m else None


def rank_diagnostics(elapsed, steps, comm_info, reducer, dev, rccl_log):
    """Collective (N > 1): per-rank step time, bucket plan / issue-order hashes, exposed comm
    time and RCCL channel count, gathered on every rank; rank 0 reports them and the order
    check has already failed the run if the ranks disagree (verify_bucket_agreement)."""
    from distributedtensorflow_amd.parallel.strategy import _digest
    plan = reducer.plan() if reducer is not None and hasattr(reducer, "plan") else None
    order = tuple(getattr(reducer, "last_order", ()))
    ch = _rccl_channels(rccl_log)
    mine = torch.tensor([elapsed / steps * 1e3, float(comm_info.get("exposed_ms_per_step", 0.0)),
                         float(len(plan["buckets"]) if plan else 0),
                         float(_digest(plan) % (1 << 52)), float(_digest(order) % (1 << 52)),
                         float(ch if ch is not None else -1)], dtype=torch.float64, device=dev)
    out = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(out, mine)
    rows = [o.tolist() for o in out]
    ms = [round(r[0], 3) for r in rows]
    return {"ms_per_step_min": min(ms), "ms_per_step_max": max(ms), "ms_per_step": ms,
            "exposed_comm_ms_per_step": [round(r[1], 3) for r in rows],
            "buckets": [int(r[2]) for r in rows],
            "plan_hash": [f"{int(r[3]):013x}" for r in rows],
            "order_hash": [f"{int(r[4]):013x}" for r in rows],
            "issue_order_rank0": list(order) if dist.get_rank() == 0 else None,
            "rccl_channels": [int(r[5]) if r[5] >= 0 else None for r in rows]}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def tuned_gemm_table(model):
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "distributedtensorflow_amd",
                        "tuning", f"tunableop_{model}.csv")


def setup_gemm_tuning(args):
    """Offline GEMM autotuning, like cuDNN's benchmark mode but ahead of time: the table maps
    each library-GEMM shape of the model to its fastest hipBLASLt solution on MI355X (measured
    once with --gemm-tuning tune; no tuning ever runs inside the timed steps)."""
    if args.gemm_tuning == "off" or args.impl != "dtf":
        return None
    import torch.cuda.tunable as tun
    if args.gemm_tuning == "tune":
        out = args.gemm_tuning_out or tuned_gemm_table(args.model)
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(20)
        tun.set_max_tuning_iterations(20)
        tun.set_filename(out, insert_device_ordinal=False)
        return out
    table = tuned_gemm_table(args.model)
    if not os.path.exists(table):
        return None
    tun.enable(True)
    tun.tuning_enable(False)
    tun.set_filename(table, insert_device_ordinal=False)
    if not tun.read_file(table):
        log(f"gemm tuning table {table} rejected (library versions differ); using defaults")
        tun.enable(False)
        return None
    return table


def build_dtf(args, dev):
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import resnet50
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import MirroredStrategy
    from distributedtensorflow_amd.train import get_or_create_global_step

    if args.strategy == "ps":
        from distributedtensorflow_amd.parallel import ParameterServerStrategy
        strategy = ParameterServerStrategy(num_ps=args.num_ps, bucket_mb=args.bucket_mb)
    else:
        strategy = MirroredStrategy(bucket_mb=args.bucket_mb)
    with strategy.scope():
        model = resnet50()
        model.train()
        # Goyal et al. recipe: lr 0.1 x (global batch / 256) after a linear warm-up
        from distributedtensorflow_amd.optimizers.optimizers import cosine_decay
        world = int(os.environ.get("WORLD_SIZE", "1"))
        lr = cosine_decay(args.lr * args.batch * world / 256, 90 * 5000, warmup_steps=500)
        opt = MomentumOptimizer(lr, momentum=0.9, weight_decay=1e-4)
        gstep = get_or_create_global_step()
        opt.build(list(model.parameters()))

    def step(images, labels):
        logits = model(images)
        loss = ops.sparse_softmax_cross_entropy(logits, labels)
        opt.minimize(loss, global_step=gstep)
        return loss

    step.optimizer = opt
    return step, strategy


def build_bert(args, dev):
    """BERT-base MLM pre-training step: MultiWorkerMirroredStrategy + fused LAMB."""
    from distributedtensorflow_amd.models.bert import bert_base
    from distributedtensorflow_amd.optimizers import LAMBOptimizer
    from distributedtensorflow_amd.optimizers.optimizers import polynomial_decay
    from distributedtensorflow_amd.parallel import MultiWorkerMirroredStrategy
    from distributedtensorflow_amd.train import get_or_create_global_step

    strategy = MultiWorkerMirroredStrategy(bucket_mb=args.bucket_mb)
    with strategy.scope():
        model = bert_base()
        model.train()
        opt = LAMBOptimizer(polynomial_decay(args.lr, 10000, warmup_steps=100),
                            weight_decay=0.01)
        gstep = get_or_create_global_step()
        opt.build(list(model.parameters()))

    def step(batch):
        loss = model(*batch)
        opt.minimize(loss, global_step=gstep)
        return loss

    step.optimizer = opt
    return step, strategy


def build_torch_bert(args, dev):
    """Stock comparator for the BERT config: HuggingFace BertForPreTraining-style MLM (random init,
    SDPA attention, bf16 autocast), fused torch AdamW (torch has no LAMB), DDP when distributed.
    The MLM head runs on the gathered masked positions only, exactly like the dtf model."""
    from transformers import BertConfig, BertForMaskedLM
    cfg = BertConfig(vocab_size=30522, hidden_size=768, num_hidden_layers=12,
                     num_attention_heads=12, intermediate_size=3072, max_position_embeddings=512,
                     attn_implementation="sdpa")
    hf = BertForMaskedLM(cfg).to(dev)

    class MaskedOnly(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, ids, seg, mask, pos):
            h = self.m.bert(input_ids=ids, token_type_ids=seg, attention_mask=mask).last_hidden_state
            hm = torch.gather(h, 1, pos.unsqueeze(-1).expand(-1, -1, h.shape[-1]))
            return self.m.cls(hm)

    model = MaskedOnly(hf).train()
    if dist.is_initialized() and dist.get_world_size() > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index],
                                                          bucket_cap_mb=args.bucket_mb)
    opt = torch.optim.AdamW(model.parameters(), lr=args.lr, weight_decay=0.01, fused=True)

    def step(batch):
        ids, seg, mask, pos, lab, _w = batch
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = model(ids, seg, mask, pos)
            loss = torch.nn.functional.cross_entropy(logits.float().flatten(0, 1), lab.flatten())
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    return step, None


def build_torch(args, dev):
    from distributedtensorflow_amd.utils.torch_baseline import TorchResNet50
    model = TorchResNet50().to(dev).to(memory_format=torch.channels_last)
    if dist.is_initialized() and dist.get_world_size() > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index],
                                                          bucket_cap_mb=args.bucket_mb)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=1e-4,
                          foreach=True)
    lossf = torch.nn.CrossEntropyLoss()

    def step(images, labels):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(images)
            loss = lossf(out.float(), labels)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    return step, None


def tune_buckets(args, opt, strategy, step, images, labels, sync, dev, steps=2):
    """All-reduce bucket size chosen by measurement (SURVEY.md 5.8 "auto-tune in the benchmark"):
    each candidate replaces the optimizer's reducer (hooks detached and re-registered), runs one
    untimed step and ``steps`` timed ones; the rank-max time decides, identically on every rank."""
    results = {}
    for mb in (16, 32, 64, 128):
        opt._reducer.close()
        strategy.bucket_bytes = int(mb * (1 << 20))
        opt._reducer = strategy.make_gradient_reducer(opt.space)
        step(images, labels)
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(images, labels)
        sync()
        t = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        results[mb] = round(float(t.item()) / steps * 1e3, 3)
    best = min(results, key=results.get)
    opt._reducer.close()
    strategy.bucket_bytes = int(best * (1 << 20))
    opt._reducer = strategy.make_gradient_reducer(opt.space)
    step(images, labels)
    sync()
    args.bucket_mb = float(best)
    return results


def fail(msg, code=2):
    print(f"bench.py: error: {msg}", file=sys.stderr, flush=True)
    sys.exit(code)


def refuse_probes():
    """Timing probes produce wrong results: a bench never runs with one requested, and never on
    a probe build of the extension (csrc: -DDTF_PROBES)."""
    bad = [k for k in os.environ if k.startswith("DTF_") and "PROBE" in k]
    if bad:
        fail(f"timing-probe variables set ({', '.join(sorted(bad))}): probes give wrong results "
             "and are never benchmarked")


def share_device():
    """``DTF_BENCH_SHARE_DEVICE=1`` (with ``DTF_BENCH_BACKEND=gloo``): every rank on cuda:0 -- the
    multi-rank rehearsal on a one-GPU box (RCCL refuses two ranks on one device)."""
    return os.environ.get("DTF_BENCH_SHARE_DEVICE", "0") == "1"


def check_devices(n):
    """Before any GPU call (``device_count`` does not initialise the GPU): N ranks need N GPUs,
    unless the gloo rehearsal shares one on purpose."""
    backend = os.environ.get("DTF_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        fail(f"DTF_BENCH_BACKEND={backend!r}: expected nccl or gloo")
    if share_device():
        if backend != "gloo":
            fail("DTF_BENCH_SHARE_DEVICE=1 needs DTF_BENCH_BACKEND=gloo (RCCL refuses two ranks "
                 "on one device)")
        if torch.cuda.device_count() < 1:
            fail("no GPU visible")
        return
    ndev = torch.cuda.device_count()
    if ndev < n:
        fail(f"--gpus {n} but only {ndev} GPU(s) are visible: refusing to measure fewer GPUs "
             f"than requested")


def _die_with_parent():
    """Child side of the fork, before exec (no GPU touched): PR_SET_PDEATHSIG = SIGKILL."""
    import ctypes
    try:
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)
    except OSError:
        pass


def self_launch(args):
    """``--gpus N`` (N > 1) without torchrun env: start the N rank processes here (one per GPU,
    torchrun's env contract: RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_*),
    stream their output through, and return the worst exit code.  When any rank fails, the
    others are terminated (they would otherwise wait in a collective for the dead one)."""
    from distributedtensorflow_amd.cluster.launcher import free_ports
    n = args.gpus
    check_devices(n)
    port = free_ports(1)[0]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(0 if share_device()
                                                                           else r),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), DTF_BENCH_LAUNCH="self")
        # same process group as this launcher (a driver's group kill reaches the ranks) and a
        # parent-death signal (a launcher killed outright takes its ranks with it)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                      env=env, cwd=ROOT, preexec_fn=_die_with_parent))
    codes = [None] * n
    failed_at = None
    try:
        while any(c is None for c in codes):
            for i, p in enumerate(procs):
                if codes[i] is None:
                    codes[i] = p.poll()
                    if codes[i] not in (None, 0) and failed_at is None:
                        failed_at = time.time()
                        print(f"bench.py: rank {i} exited with {codes[i]}; stopping the other "
                              f"ranks", file=sys.stderr, flush=True)
                        for q in procs:
                            if q.poll() is None:
                                q.send_signal(signal.SIGTERM)
            if failed_at is not None and time.time() - failed_at > 20:
                for q in procs:
                    if q.poll() is None:
                        q.kill()
            time.sleep(0.1)
    except KeyboardInterrupt:
        for q in procs:
            if q.poll() is None:
                q.kill()
        raise
    # a signal death (negative code) is a failure too
    return max(abs(c) for c in codes)


class Deadline:
    """A stack-dumping, process-ending deadline (faulthandler: a C watchdog thread that needs no
    GIL): ``arm(s)`` restarts it, ``disarm()`` cancels."""

    def arm(self, seconds, what):
        faulthandler.cancel_dump_traceback_later()
        if seconds and seconds > 0:
            self.what = what
            faulthandler.dump_traceback_later(seconds, exit=True)

    def disarm(self):
        faulthandler.cancel_dump_traceback_later()


def main():
    args = parse()
    refuse_probes()
    if args.strategy == "ps_async":
        from distributedtensorflow_amd.utils import ps_bench
        if args.job_name:
            return ps_bench.run_task(args)
        return ps_bench.run_launcher(args)
    if args.gpus < 1:
        fail("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        fail(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per requested GPU")
    if os.environ.get("DTF_BENCH_BACKEND", "nccl") == "nccl" and torch.cuda.device_count() <= local:
        fail(f"LOCAL_RANK={local} but only {torch.cuda.device_count()} GPU(s) are visible")
    deadline = Deadline()
    # one process per GPU: split the CPU quota between the node's ranks (torch's default pool is
    # sized by the whole machine and oversubscribes a shared host; see utils/cpu.py)
    from distributedtensorflow_amd.utils.cpu import usable_cpus
    per_node = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    torch.set_num_threads(max(1, usable_cpus() // max(per_node, 1)))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # DTF_FORCE_REDUCER=1 (parallel/strategy.py): a one-rank torchrun run still builds the
    # process group and the communicating reducer, so every RCCL call of the N > 1 path runs
    force = os.environ.get("DTF_FORCE_REDUCER", "0") == "1"
    rccl_log = _rccl_debug_file()
    if (world > 1 or force) and not dist.is_initialized():
        from distributedtensorflow_amd.parallel import init_process_group_from_env
        # RCCL (backend "nccl") is the measured path; DTF_BENCH_BACKEND=gloo exists only for the
        # multi-rank rehearsal on a one-GPU box (tests/test_bench_multirank_gpu.py), where RCCL
        # refuses two ranks on one device
        backend = os.environ.get("DTF_BENCH_BACKEND", "nccl")
        if backend not in ("nccl", "gloo"):
            raise SystemExit(f"DTF_BENCH_BACKEND={backend!r}: expected nccl or gloo")
        init_process_group_from_env(backend)
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)
    gemm_table = setup_gemm_tuning(args)
    native_info = {"backend": "torch (stock comparator)", "native_ext": None}
    if args.impl == "dtf":
        from distributedtensorflow_amd import ops
        from distributedtensorflow_amd.ops import native
        if ops.get_backend() == "reference":
            raise SystemExit("bench.py --impl dtf refuses DTF_OPS_BACKEND=reference: the "
                             "measured step must run this framework's HIP kernels")
        if native.kernels().probes_built():
            fail("the HIP extension is a probe build (-DDTF_PROBES): rebuild without it")
        native_info = {"backend": ops.get_backend(),
                       "native_ext": os.path.relpath(native.extension_path(), ROOT)}
    from distributedtensorflow_amd.utils import dtf_env
    native_info["dtf_env"] = dtf_env()

    # the process group that carried the gradients ("nccl" = RCCL on ROCm; None at N = 1)
    native_info["comm_backend"] = dist.get_backend() if dist.is_initialized() else None
    native_info["launch"] = {
        "mode": os.environ.get("DTF_BENCH_LAUNCH", "torchrun" if "WORLD_SIZE" in os.environ
                               else "single"),
        "env_world_size": world,
        "dist_world_size": dist.get_world_size() if dist.is_initialized() else 1,
        "rccl_version": _rccl_version(), "visible_gpus": torch.cuda.device_count(),
        "comm_timeout_s": float(os.environ.get("DTF_COMM_TIMEOUT_S", "300") or 300)}
    if native_info["launch"]["dist_world_size"] != world:
        fail(f"process group has {native_info['launch']['dist_world_size']} ranks, expected "
             f"{world}")

    strategy = None
    B, S = args.batch, args.image_size
    torch.manual_seed(1234)          # random-init weights, reproducible run to run
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    if args.model == "bert_base":
        from distributedtensorflow_amd.data.synthetic import SyntheticMLM
        if args.lr == 0.1 and "--lr" not in sys.argv:
            args.lr = 1e-3
        bert_step, strategy = (build_bert if args.impl == "dtf" else build_torch_bert)(args, dev)
        opt_for_stats = getattr(bert_step, "optimizer", None)
        d = next(iter(SyntheticMLM(B, args.seq_len, max_predictions=args.max_predictions,
                                   device=dev, seed=1234 + rank)))
        batch = (d["input_ids"], d["segment_ids"], d["input_mask"], d["masked_lm_positions"],
                 d["masked_lm_ids"], torch.ones_like(d["masked_lm_ids"], dtype=torch.float32))

        def step(_images, _labels):
            return bert_step(batch)
        images = labels = None
    elif args.impl == "dtf":
        step, strategy = build_dtf(args, dev)
        opt_for_stats = step.optimizer
        images = torch.randn(B, S, S, 3, device=dev, generator=g).to(torch.bfloat16)  # NHWC
    else:
        opt_for_stats = None
        step, _ = build_torch(args, dev)
        images = torch.randn(B, 3, S, S, device=dev, generator=g).contiguous(
            memory_format=torch.channels_last)
    if args.model != "bert_base":
        labels = torch.randint(0, 1000, (B,), device=dev, generator=g)

    def sync():
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()

    t0 = time.time()
    deadline.arm(args.warmup_timeout, "warm-up")
    for i in range(args.warmup):
        loss = step(images, labels)
    sync()
    log(f"warmup {args.warmup} steps in {time.time() - t0:.1f}s, loss={float(loss):.4f}")

    # every rank must have built the same bucket plan and issued the warm-up's bucket
    # collectives in the same order; a mismatch fails the run here (rank 0 non-zero)
    red0 = getattr(opt_for_stats, "_reducer", None)
    if dist.is_initialized() and dist.get_world_size() > 1 and hasattr(red0, "plan"):
        from distributedtensorflow_amd.parallel import verify_bucket_agreement
        try:
            verify_bucket_agreement(red0)
        except RuntimeError as e:
            fail(str(e), code=3)
    bucket_tune = None
    if args.bucket_auto and dist.is_initialized() and hasattr(getattr(opt_for_stats, "_reducer", None), "close"):
        bucket_tune = tune_buckets(args, opt_for_stats, strategy, step, images, labels, sync, dev)
        log(f"bucket auto-tune (ms/step): {bucket_tune}; using {args.bucket_mb:g} MB")
    comm = getattr(getattr(opt_for_stats, "_reducer", None), "stats", None)
    if comm is not None:
        comm.reset_timing()
        comm.timing = True
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        deadline.arm(args.step_timeout, f"timed step {i}")
        loss = step(images, labels)
    deadline.arm(2 * args.step_timeout, "final drain")
    sync()
    elapsed = time.perf_counter() - t0
    deadline.arm(args.step_timeout, "report")
    # exposed communication: compute-stream wait for RCCL after backward (0 buckets at N=1)
    comm_info = comm.as_dict() if comm is not None else {"buckets": 0,
                                                         "exposed_ms_per_step": 0.0}
    reducer = getattr(opt_for_stats, "_reducer", None)
    if reducer is not None:
        comm_info["reducer"] = type(reducer).__name__
        if hasattr(reducer, "sharded"):
            comm_info["sharded_owners"] = bool(reducer.sharded)
        if hasattr(reducer, "comm"):
            comm_info["communicator"] = reducer.comm.kind
    comm_info["forced_reducer"] = force
    if args.dump_master and opt_for_stats is not None:
        opt_for_stats.synchronize_variables()
        if rank == 0:
            torch.save(opt_for_stats.space.master.detach().cpu(), args.dump_master)
    ranks_info = None
    if dist.is_initialized() and dist.get_world_size() > 1:
        ranks_info = rank_diagnostics(elapsed, args.steps, comm_info, reducer, dev, rccl_log)
        if len(set(ranks_info["order_hash"])) > 1 or len(set(ranks_info["plan_hash"])) > 1:
            fail(f"bucket plan / issue order differs across ranks: {ranks_info}", code=3)
        comm_info["ranks"] = ranks_info
    if dist.is_initialized():
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss)
    ms = elapsed / args.steps * 1000
    ips = B * world * args.steps / elapsed
    if rank == 0 and args.model == "bert_base":
        from distributedtensorflow_amd.models.bert import BertConfig, mlm_flops_per_token
        tps = ips * args.seq_len
        fpt = mlm_flops_per_token(BertConfig(), args.seq_len, args.max_predictions)
        rec = {
            "metric": "tokens/sec (whole node) BERT-base MLM pre-training", "value": round(tps, 1),
            "unit": "tokens/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random token ids, 15% masked positions; random-init weights)",
            "config": {"model": "bert_base", "global_batch": B * world, "per_gpu_batch": B,
                       "seq_len": args.seq_len, "max_predictions": args.max_predictions,
                       "parallelism": f"dp{world}", "impl": args.impl,
                       "optimizer": "lamb+wd0.01" if args.impl == "dtf" else "torch fused AdamW+wd0.01",
                       "dropout": 0.1, "tflops_per_gpu": round(tps * fpt / world / 1e12, 1),
                       "gemm_tuning": os.path.basename(gemm_table) if gemm_table else "default",
                       "final_loss": round(final_loss, 4),
                       "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1),
                       "comm": comm_info, "bucket_mb": args.bucket_mb,
                       "bucket_tune_ms": bucket_tune, **native_info},
        }
        print(json.dumps(rec), flush=True)
    elif rank == 0:
        rec = {
            "metric": METRIC, "value": round(ips, 2), "unit": "images/sec",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": (round(ips / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            "dtype": "bf16", "data": "synthetic (random NHWC 224x224x3 images, random labels; "
                                      "random-init weights)",
            "config": {"model": "resnet50", "global_batch": B * world, "per_gpu_batch": B,
                       "seq_len": None, "image_size": S,
                       "parallelism": (f"dp{world}" if args.strategy == "mirrored" else
                                       f"ps{min(args.num_ps, world)}+dp{world}"),
                       "impl": args.impl, "optimizer": "momentum0.9+wd1e-4, lr 0.1*B/256 warmup500+cosine",
                       "cudnn_benchmark": bool(args.cudnn_benchmark) if args.impl == "torch" else None,
                       "final_loss": round(final_loss, 4),
                       "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1),
                       "comm": comm_info, "bucket_mb": args.bucket_mb,
                       "bucket_tune_ms": bucket_tune, **native_info},
        }
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    deadline.disarm()


if __name__ == "__main__":
    main()
    # the run is done and reported (its process group destroyed in main): leave without the
    # interpreter's teardown, where a C++ runtime thread raced the static destructors once on the
    # 2-rank gloo rehearsal ("terminate called without an active exception" after the JSON line,
    # test_bench_self_launches_n_ranks_without_torchrun, profiles/r6)
    # (ranks of a multi-rank job only: a single process keeps its normal exit, which profilers
    # such as rocprofv3 need to write their output)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
