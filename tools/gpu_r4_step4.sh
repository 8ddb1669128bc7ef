# Round 4: pipelined-PS determinism test, ps_async 2-worker bench, kernel profiles of both benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_ps_gpu.py -k "pipelined" > gpurun_out/r4_t3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --strategy ps_async --num-workers 2 > gpurun_out/r4_bench_psasync2.json 2> gpurun_out/r4_bench_psasync2.err || exit 1
timeout -k 10 200 python bench.py > gpurun_out/r4_bench_resnet_mirrored.json 2> gpurun_out/r4_bench_resnet_mirrored.err || exit 1
PROF_NAME=r4_resnet SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh || exit 1
PROF_NAME=r4_bert SKIP_TORCH=1 DTF_BENCH_ARGS="--model bert_base" bash tools/prof_bench.sh
