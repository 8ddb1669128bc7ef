#!/bin/bash
# row-streaming GEMM v2 (swapped operands, 8-B staging, statistics from the read-back): tests + timing
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3r
timeout -k 10 300 python -u -m pytest tests/test_gemm_stream_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3r/pytest_stream.log 2>&1 || { tail -40 gpurun_out/r3r/pytest_stream.log; exit 1; }
tail -2 gpurun_out/r3r/pytest_stream.log
timeout -k 10 300 python -u tools/gemm_bench.py --shapes 388864x1024x256,1555456x512x128,6221824x256x64,6221824x64x64 --variants 13 --dbg 0,1,2,15,0 --iters 10 --out gpurun_out/r3r/stream_probe.jsonl > gpurun_out/r3r/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3r/gemm_bench.log; exit 1; }
timeout -k 10 400 python -u tools/gemm_bench.py --resnet1x1 1984 --variants 13 --iters 10 > gpurun_out/r3r/resnet1x1.log 2>&1 || { tail -30 gpurun_out/r3r/resnet1x1.log; exit 1; }
