#!/bin/bash
# native RCCL communicator tests, then the b1024 same-box comparator
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/r3i
timeout -k 10 300 python -u -m pytest tests/test_rccl_comm_gpu.py tests/test_forced_reducer_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r3i/pytest_rccl.log 2>&1 || { tail -40 gpurun_out/r3i/pytest_rccl.log; exit 1; }
tail -12 gpurun_out/r3i/pytest_rccl.log
BATCH=1024 bash tools/comparator.sh
