#!/bin/bash
# One measure iteration on the GPU box: targeted kernel tests, micro-benches, bench + profile.
#   STEPS="kernels bn bench prof" bash tools/gpu_iter.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/iter"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONPATH="$R"
for s in ${STEPS:-kernels bn bench prof}; do
  case $s in
    kernels) timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_resnet_gpu.py \
               -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1 || exit $? ;;
    gputests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $? ;;
    bn) timeout -k 10 300 python -u tools/bn_bench.py --out "$OUT/bn_bandwidth_b512.jsonl" > "$OUT/bn_bench.log" 2>&1 || exit $? ;;
    conv) timeout -k 10 400 python -u tools/conv_bench.py ${CONV_ARGS} > "$OUT/conv_bench.log" 2>&1 || exit $? ;;
    bench) timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_resnet.log" 2>&1 || exit $? ;;
    bert) timeout -k 10 300 python -u bench.py --model bert_base --steps 20 --warmup 5 > "$OUT/bench_bert.log" 2>&1 || exit $? ;;
    smoke) timeout -k 10 300 python -u __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || exit $? ;;
    prof) SKIP_TORCH=1 PROF_NAME=iter timeout -k 10 700 bash tools/prof_bench.sh || exit $? ;;
    bertprof) SKIP_TORCH=1 PROF_NAME=bert DTF_BENCH_ARGS="--model bert_base" timeout -k 10 700 bash tools/prof_bench.sh || exit $? ;;
  esac
  echo "step $s ok"
done
