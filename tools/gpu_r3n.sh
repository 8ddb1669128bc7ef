#!/bin/bash
# round-3 HEAD evidence: conv roofline at b1984, rocprof kernel summaries of the ResNet-50 and
# BERT-base steps, PMC counters of the weakest conv shapes
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3n
timeout -k 10 400 python -u tools/conv_bench.py --batch 1984 --iters 10 > gpurun_out/r3n/conv_roofline_b1984.log 2>&1 || { tail -20 gpurun_out/r3n/conv_roofline_b1984.log; exit 1; }
SKIP_TORCH=1 PROF_NAME=r3_resnet bash tools/prof_bench.sh || exit $?
SKIP_TORCH=1 PROF_NAME=r3_bert DTF_BENCH_ARGS="--model bert_base" bash tools/prof_bench.sh || exit $?
LAYERS=s1b1c2,s2b0c2,s3b0c2,s1b0c2,s3b1c1,s3b0c3 bash tools/pmc_conv.sh || exit $?
