#!/bin/bash
# per-GPU batch sweep of the ResNet-50 bench (tile-count quantization vs 256 CUs)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/bs
for b in ${BATCHES:-512 576 640 768}; do
  timeout -k 10 300 python -u bench.py --batch $b --steps 20 --warmup 5 > gpurun_out/bs/b$b.log 2>&1 || exit $?
done
