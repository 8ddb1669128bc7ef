#!/bin/bash
# Same-box A/B of the bench under env switches: AB="VAR=a VAR=b ..." (one run each);
# BENCH_ARGS="--model bert_base" for BERT
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/ab
i=0
for kv in ${AB}; do
  i=$((i+1))
  env $kv timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/ab/run$i.log 2>&1 || exit $?
  echo "$kv $(tail -1 gpurun_out/ab/run$i.log | cut -c1-140)" >> gpurun_out/ab/summary.txt
done
