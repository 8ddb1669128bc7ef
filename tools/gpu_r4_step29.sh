# Round 4: BERT FFN1 forward on our GEMM with the bias + GELU epilogue: numerics, kernel timings,
# BERT-base A/B (DTF_FFN_GEMM_GELU).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nlp.py -k "gelu or bert" > gpurun_out/r4_t29.log 2>&1 || exit 1
timeout -k 10 120 python tools/gelu_gemm_bench.py > gpurun_out/r4_ffn1_fused.jsonl 2> gpurun_out/r4_ffn1_fused.err || exit 1
for v in 1 0 1 0; do
  DTF_FFN_GEMM_GELU=$v timeout -k 10 240 python bench.py --model bert_base > gpurun_out/r4_bert_ffn_$v.json 2> gpurun_out/r4_bert_ffn_$v.err || exit 1
  cat gpurun_out/r4_bert_ffn_$v.json >> gpurun_out/r4_bert_ffn1_fused_ab.jsonl
done
