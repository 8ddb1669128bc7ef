#!/bin/bash
# row-streaming GEMM: bit-identity tests, 1x1 shapes vs the conv kernel, ResNet-50 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3p
timeout -k 10 300 python -u -m pytest tests/test_gemm_stream_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3p/pytest_stream.log 2>&1 || { tail -40 gpurun_out/r3p/pytest_stream.log; exit 1; }
tail -3 gpurun_out/r3p/pytest_stream.log
timeout -k 10 400 python -u tools/gemm_bench.py --resnet1x1 1984 --variants 8,13 --iters 10 --out gpurun_out/r3p/resnet1x1.jsonl > gpurun_out/r3p/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3p/gemm_bench.log; exit 1; }
for i in 1 2; do
  DTF_GEMM_STREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3p/bench_off_$i.log 2>&1 || { tail -20 gpurun_out/r3p/bench_off_$i.log; exit 1; }
  DTF_GEMM_STREAM=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3p/bench_on_$i.log 2>&1 || { tail -20 gpurun_out/r3p/bench_on_$i.log; exit 1; }
done
grep -h '^{' gpurun_out/r3p/bench_*.log | cut -c1-200
