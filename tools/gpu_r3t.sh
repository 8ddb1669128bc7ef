#!/bin/bash
# row-streaming GEMM with compile-time modes / waits: tests, 1x1 shapes, ResNet-50 bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3t
timeout -k 10 300 python -u -m pytest tests/test_gemm_stream_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3t/pytest_stream.log 2>&1 || { tail -40 gpurun_out/r3t/pytest_stream.log; exit 1; }
tail -2 gpurun_out/r3t/pytest_stream.log
timeout -k 10 300 python -u tools/gemm_bench.py --shapes 388864x1024x256,1555456x512x128,6221824x256x64,6221824x64x64 --variants 13 --iters 10 --out gpurun_out/r3t/stream.jsonl > gpurun_out/r3t/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3t/gemm_bench.log; exit 1; }
timeout -k 10 400 python -u tools/gemm_bench.py --resnet1x1 1984 --variants 13 --iters 10 > gpurun_out/r3t/resnet1x1.log 2>&1 || { tail -30 gpurun_out/r3t/resnet1x1.log; exit 1; }
for i in 1 2; do
  DTF_GEMM_STREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3t/bench_off_$i.log 2>&1 || { tail -20 gpurun_out/r3t/bench_off_$i.log; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3t/bench_on_$i.log 2>&1 || { tail -20 gpurun_out/r3t/bench_on_$i.log; exit 1; }
done
