# Round 4: projection-block (dual BN) d(c3 output) formed in the fused c3 backward too.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/r4_t7.log 2>&1 || exit 1
DTF_FUSE_C3_LAZY=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lzd1.json 2> gpurun_out/r4_bench_lzd1.err || exit 1
DTF_FUSE_C3_LAZY=0 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lzd0.json 2> gpurun_out/r4_bench_lzd0.err || exit 1
DTF_FUSE_C3_LAZY=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lzd1b.json 2> gpurun_out/r4_bench_lzd1b.err
