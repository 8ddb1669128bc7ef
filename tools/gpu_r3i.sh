# stock PyTorch-ROCm comparator at the bench batch (1984) with MIOpen's fast find mode, next to
# this framework on the same box
cd $GRAFT_REPO_ROOT || exit 1
export PYTHONPATH=$PWD
mkdir -p gpurun_out/r3i
( while true; do date >> gpurun_out/r3i/heartbeat.txt; sleep 45; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3i/bench_dtf_b1984.log 2>&1 &&
MIOPEN_FIND_MODE=FAST timeout -k 10 900 python -u bench.py --impl torch --batch 1984 --cudnn-benchmark 0 --steps 10 --warmup 3 > gpurun_out/r3i/bench_torch_b1984_fast.log 2>&1
