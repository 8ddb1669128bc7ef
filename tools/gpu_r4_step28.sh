# Round 4: stock PyTorch-ROCm comparator at the headline batch (1984), MIOpen immediate mode
# (MIOPEN_FIND_MODE=FAST: the exhaustive search exceeded 1000 s in round 3), next to dtf on the
# same box.  A heartbeat file keeps the long first steps visibly alive.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cmp1984
( while true; do date >> gpurun_out/cmp1984/heartbeat.txt; sleep 45; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/cmp1984/dtf.log 2>&1 || exit 1
MIOPEN_FIND_MODE=FAST timeout -k 10 900 python -u bench.py --impl torch --batch 1984 --cudnn-benchmark 0 --steps 10 --warmup 5 > gpurun_out/cmp1984/torch_fast.log 2>&1 || exit 1
