# Round 4: GELU-backward GEMM epilogue with its GELU-input loads up front: kernel timing, numerics,
# BERT-base A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python tools/gelu_gemm_bench.py > gpurun_out/r4_gelu_gemm.jsonl 2> gpurun_out/r4_gelu_gemm.err || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nlp.py tests/test_dense_gpu.py -k "gelu or bert or dense" > gpurun_out/r4_t23.log 2>&1 || exit 1
for v in 1 0 1 0; do
  DTF_GEMM_GELU_PRE=$v timeout -k 10 240 python bench.py --model bert_base > gpurun_out/r4_bert_gpre_$v.json 2> gpurun_out/r4_bert_gpre_$v.err || exit 1
  cat gpurun_out/r4_bert_gpre_$v.json >> gpurun_out/r4_bert_gelu_pre_ab.jsonl
done
