# Round 4: GEMM epilogue extra-input loads up front (GELU input, accumulate source, masked residual
# gradient; dense GEMMs): numerics, kernel timing, BERT-base and ResNet-50 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nlp.py tests/test_dense_gpu.py tests/test_gemm_pp_gpu.py tests/test_kernels_gpu.py tests/test_resnet_gpu.py -m gpu -k "gelu or bert or dense or gemm or direct_grad or lazy or teacher or residual" > gpurun_out/r4_t24.log 2>&1 || exit 1
timeout -k 10 120 python tools/gelu_gemm_bench.py > gpurun_out/r4_gelu_gemm2.jsonl 2> gpurun_out/r4_gelu_gemm2.err || exit 1
for v in 1 0 1 0; do
  DTF_GEMM_GELU_PRE=$v timeout -k 10 240 python bench.py --model bert_base > gpurun_out/r4_bert_pre2_$v.json 2> gpurun_out/r4_bert_pre2_$v.err || exit 1
  cat gpurun_out/r4_bert_pre2_$v.json >> gpurun_out/r4_bert_epi_pre_ab.jsonl
done
for v in 1 0 1 0; do
  DTF_GEMM_GELU_PRE=$v timeout -k 10 200 python bench.py > gpurun_out/r4_rn_pre2_$v.json 2> gpurun_out/r4_rn_pre2_$v.err || exit 1
  cat gpurun_out/r4_rn_pre2_$v.json >> gpurun_out/r4_resnet_epi_pre_ab.jsonl
done
