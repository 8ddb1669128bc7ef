#!/bin/bash
# Full GPU verification pass: every gpu-marked test, smoke(), ResNet-50 + BERT benches.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/check"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONPATH="$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_resnet.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --model bert_base --steps 20 --warmup 5 > "$OUT/bench_bert.log" 2>&1 || exit $?
