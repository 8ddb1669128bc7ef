#!/bin/bash
# full GPU suite + smoke + default bench at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3ab
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3ab/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r3ab/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r3ab/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ab/smoke.log 2>&1 || { tail -20 gpurun_out/r3ab/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r3ab/bench.log 2>&1 || { tail -20 gpurun_out/r3ab/bench.log; exit 1; }
grep '^{' gpurun_out/r3ab/bench.log | cut -c1-300
