#!/bin/bash
# re-measure the 4-wave 128x128-wave-tile GEMM variants (5, 6, 7) against the ping-pong (8)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3k
timeout -k 10 300 python -u tools/gemm_bench.py --variants 8,5,6,7 --iters 20 --only bert_qkv_fwd,bert_attnout_fwd,bert_ffn1_fwd,bert_ffn2_fwd,sq8192 --out gpurun_out/r3k/gemm_nw4.jsonl > gpurun_out/r3k/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3k/gemm_bench.log; exit 1; }
