#!/bin/bash
# dtf vs the stock PyTorch-ROCm comparator at the same per-GPU batch.  MIOpen's first-call
# algorithm search makes the comparator's first steps silent for minutes: a heartbeat file keeps
# the run visibly alive (each step is still bounded by its own timeout).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/cmp
B=${BATCH:-1024}
( while true; do date >> gpurun_out/cmp/heartbeat.txt; sleep 45; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u bench.py --batch $B --steps 20 --warmup 5 > gpurun_out/cmp/dtf_b$B.log 2>&1 || exit $?
timeout -k 10 1000 python -u bench.py --impl torch --batch $B --steps 20 --warmup 15 > gpurun_out/cmp/torch_b$B.log 2>&1 || exit $?
