# Round 4 (final tree): full GPU suite, smoke, default 1-GPU bench, BERT bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_final.log 2>&1 || { tail -30 gpurun_out/r4_pytest_gpu_final.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/r4_smoke_final.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r4_bench_final.json 2> gpurun_out/r4_bench_final.err || exit 1
timeout -k 10 300 python bench.py --model bert_base > gpurun_out/r4_bench_bert_final.json 2> gpurun_out/r4_bench_bert_final.err || exit 1
