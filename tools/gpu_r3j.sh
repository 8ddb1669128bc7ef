#!/bin/bash
# OCC-2 256x128 GEMM (variant 12): bit-identity vs variant 8, then timing vs 8 and hipBLASLt
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3j
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -x -q --timeout 120 --timeout-method thread -k "12" > gpurun_out/r3j/pytest_v12.log 2>&1 || { tail -30 gpurun_out/r3j/pytest_v12.log; exit 1; }
tail -3 gpurun_out/r3j/pytest_v12.log
timeout -k 10 400 python -u tools/gemm_bench.py --variants 8,12 --stagger 1:-1,0:0,2:-1,3:-1,1:1,1:6 --iters 20 --out gpurun_out/r3j/gemm_v12.jsonl > gpurun_out/r3j/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3j/gemm_bench.log; exit 1; }
