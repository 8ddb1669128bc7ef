#!/bin/bash
# A/B: BERT dense weight gradients up to 3072 x 768 (the FFN layers too) on our TN wgrad kernel
# vs the round-3 cap of 2304 x 768 (FFN weight gradients on hipBLASLt), alternating, same box
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for i in 1 2; do
  for cap in 2359296 1769472; do
    DTF_DENSE_WGRAD_NATIVE_MAX=$cap timeout -k 10 300 python -u bench.py --model bert_base --steps 20 --warmup 5 > gpurun_out/bwc_${cap}_$i.log 2>&1 || exit 1
    grep '^{' gpurun_out/bwc_${cap}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('cap', $cap, d['value'], d['ms_per_step'])"
  done
done
