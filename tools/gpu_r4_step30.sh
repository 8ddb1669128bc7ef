# Round 4: BERT kernel profiles with the FFN1 fused bias + GELU GEMM on and off (why the faster op
# loses in the step).
set -o pipefail
cd $GRAFT_REPO_ROOT
DTF_FFN_GEMM_GELU=1 PROF_NAME=r4_bert_ffn1_on SKIP_TORCH=1 DTF_BENCH_ARGS="--model bert_base" bash tools/prof_bench.sh || exit 1
DTF_FFN_GEMM_GELU=0 PROF_NAME=r4_bert_ffn1_off SKIP_TORCH=1 DTF_BENCH_ARGS="--model bert_base" bash tools/prof_bench.sh
