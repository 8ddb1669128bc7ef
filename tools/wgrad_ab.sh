#!/bin/bash
# A/B of the wgrad kernel variants on the Kout <= 64 layers (narrow 1x4 vs 2x2 LDS-DMA)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=. && mkdir -p gpurun_out/wab
for m in 1 2; do
  timeout -k 10 300 python -u tools/conv_bench.py --kinds wgrad --wgrad-mode $m \
    --only stem_s2d,s0b0c1,s0b0c2,s0b1c1,s0b0c3 > gpurun_out/wab/m$m.log 2>&1 || exit $?
done
