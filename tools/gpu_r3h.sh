# full GPU verification + the stock comparator on the same box (round 3)
cd $GRAFT_REPO_ROOT || exit 1
export PYTHONPATH=$PWD
mkdir -p gpurun_out/r3h
( while true; do date >> gpurun_out/r3h/heartbeat.txt; sleep 45; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r3h/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/r3h/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3h/bench_dtf_b1984.log 2>&1 &&
timeout -k 10 420 python -u bench.py --impl torch --batch 1984 --cudnn-benchmark 0 --steps 10 --warmup 5 > gpurun_out/r3h/bench_torch_b1984_immediate.log 2>&1
