# Round 4: stage-0 lazy d(c3 output) with x3 recomputed (RC): numerics + A/B (stage-0 RC vs round
# state before it is not a knob; compare DTF_FUSE_C3_LAZY on/off on the same box).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/r4_t10.log 2>&1 || exit 1
DTF_FUSE_C3_LAZY=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_rc1.json 2> gpurun_out/r4_bench_rc1.err || exit 1
DTF_FUSE_C3_LAZY=0 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_rc0.json 2> gpurun_out/r4_bench_rc0.err || exit 1
DTF_FUSE_C3_LAZY=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_rc1b.json 2> gpurun_out/r4_bench_rc1b.err || exit 1
PROF_NAME=r4_resnet_v3 SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh
