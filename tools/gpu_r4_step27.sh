# Round 4 (late): the full GPU suite, smoke, the default 1-GPU bench, and the BERT v3 profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_pytest_gpu_full2.log 2>&1 || { tail -30 gpurun_out/r4_pytest_gpu_full2.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/r4_smoke2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r4_bench_default.json 2> gpurun_out/r4_bench_default.err || exit 1
PROF_NAME=r4_bert_v3 SKIP_TORCH=1 DTF_BENCH_ARGS="--model bert_base" bash tools/prof_bench.sh
