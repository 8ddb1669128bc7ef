set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_resnet_gpu.py -k "bn or batch or resnet" > gpurun_out/ab_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -3 gpurun_out/ab_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_new_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab_new_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('new', d['value'], d['ms_per_step'])"
  DTF_BN_GRID_CAP=2048 DTF_BN_STATS_BLOCKS=1024 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_old_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab_old_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('old', d['value'], d['ms_per_step'])"
done
