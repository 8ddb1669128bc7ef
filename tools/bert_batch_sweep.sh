#!/bin/bash
# per-GPU batch sweep of the BERT-base MLM bench (seq 128)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/bbs
for b in ${BATCHES:-128 256 512}; do
  timeout -k 10 300 python -u bench.py --model bert_base --batch $b --steps 20 --warmup 5 > gpurun_out/bbs/b$b.log 2>&1 || exit $?
done
