# Round 4: dual-BN sums in the streamed c1 data gradient: numerics, then A/B on the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet_gpu.py tests/test_gemm_stream_gpu.py > gpurun_out/r4_t5.log 2>&1 || exit 1
DTF_FUSE_DUAL_BNB=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_resnet_dual1.json 2> gpurun_out/r4_bench_resnet_dual1.err || exit 1
DTF_FUSE_DUAL_BNB=0 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_resnet_dual0.json 2> gpurun_out/r4_bench_resnet_dual0.err || exit 1
DTF_FUSE_DUAL_BNB=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_resnet_dual1b.json 2> gpurun_out/r4_bench_resnet_dual1b.err
