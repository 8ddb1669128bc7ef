#!/bin/bash
# where the ping-pong GEMM's epilogue time goes: dbg 1 = no epilogue, 2 = no C stores, 4 = no LDS staging
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3l
timeout -k 10 300 python -u tools/gemm_bench.py --variants 8 --dbg 0,1,2,4,6,0 --iters 30 --only bert_qkv_fwd,bert_attnout_fwd,bert_ffn1_fwd,bert_ffn2_dgrad --out gpurun_out/r3l/gemm_epi.jsonl > gpurun_out/r3l/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3l/gemm_bench.log; exit 1; }
