set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SH=bert_qkv_fwd,bert_attnout_fwd,bert_ffn1_fwd,bert_ffn2_fwd,bert_qkv_dgrad,bert_ffn1_dgrad,bert_ffn2_dgrad
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nlp.py -k "attention or qkv_bias or mlm or gelu_dense" > gpurun_out/r4_t0.log 2>&1 || exit 1
for gm in 0 4 8 16; do
  DTF_GEMM_GROUP_M=$gm timeout -k 10 120 python tools/gemm_bench.py --only $SH --iters 20 --variants 8 --out gpurun_out/r4_gemm_group_$gm.jsonl > gpurun_out/r4_gemm_group_$gm.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --model bert_base > gpurun_out/r4_bench_bert.json 2> gpurun_out/r4_bench_bert.err && \
DTF_ATTN_FUSED_BWD=0 timeout -k 10 200 python bench.py --model bert_base > gpurun_out/r4_bench_bert_split.json 2> gpurun_out/r4_bench_bert_split.err && \
timeout -k 10 200 python bench.py > gpurun_out/r4_bench_resnet.json 2> gpurun_out/r4_bench_resnet.err && \
timeout -k 10 500 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_recovery_gpu.py tests/test_bench_multirank_gpu.py tests/test_ps_gpu.py > gpurun_out/r4_t1.log 2>&1 && \
timeout -k 10 300 python bench.py --strategy ps_async --num-workers 2 > gpurun_out/r4_bench_psasync2.json 2> gpurun_out/r4_bench_psasync2.err
[ $? -eq 0 ] || exit 1
PROF_NAME=r4_bert SKIP_TORCH=1 DTF_BENCH_ARGS="--model bert_base" bash tools/prof_bench.sh && \
PROF_NAME=r4_resnet SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh
