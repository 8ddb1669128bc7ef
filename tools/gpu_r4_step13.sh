# Round 4: stage-0 fused c3 backward as 16-wave blocks: kernel timings, numerics, ResNet A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 180 python tools/c1_bench.py > gpurun_out/r4_c1_bench_w16.jsonl 2> gpurun_out/r4_c1_bench_w16.err || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet_gpu.py -k "lazy or fused_c1" > gpurun_out/r4_t13.log 2>&1 || exit 1
for v in 1 0 1 0; do
  DTF_C1_W16=$v timeout -k 10 200 python bench.py > gpurun_out/r4_bench_w16_$v.json 2> gpurun_out/r4_bench_w16_$v.err || exit 1
  cp gpurun_out/r4_bench_w16_$v.json gpurun_out/r4_bench_w16_${v}_$(date +%s%N).json
done
