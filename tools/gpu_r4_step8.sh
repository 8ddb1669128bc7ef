# Round 4: the whole GPU test suite, smoke(), and a kernel profile of the current ResNet-50 step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r4_gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || exit 1
PROF_NAME=r4_resnet_v2 SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh
