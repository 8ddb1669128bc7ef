#!/bin/bash
# ResNet-50 1x1 convs at b1984 as GEMMs: ping-pong (8) vs two-blocks-per-CU 256x128 (12) vs the conv kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3o
timeout -k 10 400 python -u tools/gemm_bench.py --resnet1x1 1984 --variants 8,12,1 --iters 10 --out gpurun_out/r3o/resnet1x1.jsonl > gpurun_out/r3o/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3o/gemm_bench.log; exit 1; }
