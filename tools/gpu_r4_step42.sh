# Round 4: stride-2 dgrad BN sums on by default for the 128-output dgrad: ResNet GPU tests and the
# kernel profile (bn_reduce per step).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_gemm_stream_gpu.py > gpurun_out/r4_t42.log 2>&1 || { tail -20 gpurun_out/r4_t42.log; exit 1; }
PROF_NAME=r4_resnet_v6 SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh
