#!/bin/bash
# One GPU session of headline measurements (each step time-limited, chained).
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/measure"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONPATH="$R"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > "$OUT/bench_resnet_b512.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --model bert_base --steps 20 --warmup 5 > "$OUT/bench_bert.log" 2>&1 || exit $?
( time timeout -k 10 400 python -m distributedtensorflow_amd.cluster.launcher run_mnist_distributed.py \
    --num_ps 1 --num_workers 2 --workdir /tmp/mnist_gpu --max_steps 1000 --data_dir /tmp/mnist_gpu_data \
    --log_dir /tmp/mnist_gpu/tb ) > "$OUT/mnist_ps_gpu.log" 2>&1 || exit $?
tail -3 /tmp/mnist_gpu/worker0.log >> "$OUT/mnist_ps_gpu.log"
tail -1 /tmp/mnist_gpu/ps0.log >> "$OUT/mnist_ps_gpu.log"
timeout -k 10 900 python bench.py --impl torch --steps 30 --warmup 15 > "$OUT/bench_torch_b512.log" 2>&1 || exit $?
