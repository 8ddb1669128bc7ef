# Round 4: fused c3 backward kernel timings (tools/c1_bench.py), lazy numerics, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python tools/c1_bench.py > gpurun_out/r4_c1_bench.jsonl 2> gpurun_out/r4_c1_bench.err || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet_gpu.py -k "lazy or fused_c1" > gpurun_out/r4_t11.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/r4_bench_v11.json 2> gpurun_out/r4_bench_v11.err
