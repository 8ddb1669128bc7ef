# Round 4: stage-1 lazy d(c3 output) and the two-blocks-per-CU attention backward: numerics +
# A/B, then the whole GPU suite, smoke, profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resnet_gpu.py tests/test_nlp.py > gpurun_out/r4_t9.log 2>&1 || exit 1
DTF_FUSE_C3_LAZY=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lzs1.json 2> gpurun_out/r4_bench_lzs1.err || exit 1
DTF_FUSE_C3_LAZY=0 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lzs0.json 2> gpurun_out/r4_bench_lzs0.err || exit 1
DTF_FUSE_C3_LAZY=1 timeout -k 10 200 python bench.py > gpurun_out/r4_bench_lzs1b.json 2> gpurun_out/r4_bench_lzs1b.err || exit 1
timeout -k 10 200 python bench.py --model bert_base > gpurun_out/r4_bench_bert_f2.json 2> gpurun_out/r4_bench_bert_f2.err || exit 1
DTF_ATTN_FUSED_BWD=0 timeout -k 10 200 python bench.py --model bert_base > gpurun_out/r4_bench_bert_s2.json 2> gpurun_out/r4_bench_bert_s2.err || exit 1
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/r4_attn_bench.jsonl 2> gpurun_out/r4_attn_bench.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r4_gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || exit 1
PROF_NAME=r4_resnet_v2 SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh
