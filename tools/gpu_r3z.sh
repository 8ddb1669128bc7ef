#!/bin/bash
# BN + ReLU inside c3's streaming GEMM: tests + ResNet-50 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3z
timeout -k 10 500 python -u -m pytest tests/test_gemm_stream_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3z/pytest.log 2>&1 || { tail -50 gpurun_out/r3z/pytest.log; exit 1; }
tail -2 gpurun_out/r3z/pytest.log
for i in 1 2; do
  DTF_FUSE_BN_CONV=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3z/bench_off_$i.log 2>&1 || { tail -20 gpurun_out/r3z/bench_off_$i.log; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3z/bench_on_$i.log 2>&1 || { tail -20 gpurun_out/r3z/bench_on_$i.log; exit 1; }
done
