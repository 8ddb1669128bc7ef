#!/bin/bash
# full GPU suite + smoke + profile of the ResNet-50 step at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3u
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3u/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r3u/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r3u/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3u/smoke.log 2>&1 || { tail -20 gpurun_out/r3u/smoke.log; exit 1; }
SKIP_TORCH=1 PROF_NAME=r3u_resnet bash tools/prof_bench.sh || exit $?
