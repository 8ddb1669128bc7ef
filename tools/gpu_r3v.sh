#!/bin/bash
# BERT dW: hipBLASLt split-K + slab sum vs the native TN wgrad kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3v
timeout -k 10 300 python -u tools/dense_wgrad_bench.py --iters 10 --out gpurun_out/r3v/dense_wgrad.jsonl > gpurun_out/r3v/dense_wgrad.log 2>&1 || { tail -30 gpurun_out/r3v/dense_wgrad.log; exit 1; }
