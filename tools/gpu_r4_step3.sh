# Round 4: fused first-stage c3 backward (conv1x1_bwd.hip) numerics + A/B, the recovery / PS /
# self-launch GPU tests, then kernel profiles of both benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_resnet_gpu.py -k "fused_c1" > gpurun_out/r4_c1.log 2>&1 || exit 1
DTF_FUSE_C1_BWD=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_resnet_c1.json 2> gpurun_out/r4_bench_resnet_c1.err || exit 1
DTF_FUSE_C1_BWD=0 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_resnet_noc1.json 2> gpurun_out/r4_bench_resnet_noc1.err || exit 1
DTF_GEMM_GROUP_M=8 timeout -k 10 200 python bench.py --model bert_base > gpurun_out/r4_bench_bert_g8.json 2> gpurun_out/r4_bench_bert_g8.err || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_resnet_gpu.py tests/test_recovery_gpu.py tests/test_bench_multirank_gpu.py tests/test_ps_gpu.py > gpurun_out/r4_t2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --strategy ps_async --num-workers 2 > gpurun_out/r4_bench_psasync2.json 2> gpurun_out/r4_bench_psasync2.err || exit 1
PROF_NAME=r4_resnet SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh || exit 1
PROF_NAME=r4_bert SKIP_TORCH=1 DTF_BENCH_ARGS="--model bert_base" bash tools/prof_bench.sh
