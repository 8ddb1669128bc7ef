# Round 4: residual-BN d(c3 output) formed inside the fused c3 backward (LZ): numerics + A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/r4_t6.log 2>&1 || exit 1
DTF_FUSE_C3_LAZY=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lz1.json 2> gpurun_out/r4_bench_lz1.err || exit 1
DTF_FUSE_C3_LAZY=0 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lz0.json 2> gpurun_out/r4_bench_lz0.err || exit 1
DTF_FUSE_C3_LAZY=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lz1b.json 2> gpurun_out/r4_bench_lz1b.err || exit 1
DTF_FUSE_C3_LAZY=0 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lz0b.json 2> gpurun_out/r4_bench_lz0b.err
