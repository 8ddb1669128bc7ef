#!/bin/bash
# first-round start stagger of the ping-pong GEMM (stagger_mode 4): do de-phased tile rounds spread the C-store bursts?
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3m
timeout -k 10 300 python -u tools/gemm_bench.py --variants 8 --iters 30 --stagger-occ1 0:0,4:1,4:2,4:3,0:0 --only bert_qkv_fwd,bert_attnout_fwd,bert_ffn1_fwd,bert_ffn2_dgrad,bert_ffn2_fwd --out gpurun_out/r3m/gemm_stagger.jsonl > gpurun_out/r3m/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3m/gemm_bench.log; exit 1; }
