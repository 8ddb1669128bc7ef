#!/bin/bash
# A/B: conv weight gradients on a side stream (DTF_WGRAD_SIDE=1) vs in line, ResNet-50 b1984
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
DTF_WGRAD_SIDE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_resnet_gpu.py > gpurun_out/side_tests.log 2>&1 || { tail -30 gpurun_out/side_tests.log; exit 1; }
tail -2 gpurun_out/side_tests.log
for i in 1 2; do
  for mode in 1 0; do
    DTF_WGRAD_SIDE=$mode timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/side_${mode}_$i.log 2>&1 || exit 1
    grep '^{' gpurun_out/side_${mode}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('side', $mode, d['value'], d['ms_per_step'], d['config'].get('final_loss'), d['config'].get('peak_mem_gb'))"
  done
done
