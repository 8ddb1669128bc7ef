#!/bin/bash
# GEMM kernel check on the GPU box: numerics / bit-identity tests, epilogue overhead probe,
# BERT-shape comparison with hipBLASLt.  Results under gpurun_out/gemm/.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/gemm"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONPATH="$R"
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_overhead.py --N 768 --K 256,768,3072 --out "$OUT/overhead.jsonl" > "$OUT/overhead.log" 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_bench.py --variants=-1 --out "$OUT/gemm_bench.jsonl" > "$OUT/gemm_bench.log" 2>&1 || exit $?
