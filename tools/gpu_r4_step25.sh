# Round 4: same-box comparison of the GEMM epilogue prefetch against the round-3 epilogue
# (-DDTF_GEMM_EPI_LEGACY build, made on the box): GELU-backward GEMM timing and BERT-base.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # tag
  timeout -k 10 120 python tools/gelu_gemm_bench.py | sed "s/^{/{\"build\": \"$1\", /" >> gpurun_out/r4_epi_legacy_gemm.jsonl || return 1
  for i in 1 2; do
    timeout -k 10 240 python bench.py --model bert_base > gpurun_out/r4_epi_$1_$i.json 2> gpurun_out/r4_epi_$1_$i.err || return 1
    sed "s/^{/{\"build\": \"$1\", /" gpurun_out/r4_epi_$1_$i.json >> gpurun_out/r4_epi_legacy_bert.jsonl
  done
}
run new || exit 1
DTF_HIP_EXTRA_FLAGS=-DDTF_GEMM_EPI_LEGACY timeout -k 10 600 python -c "from distributedtensorflow_amd import _build; _build.build_all()" > gpurun_out/r4_epi_legacy_build.log 2>&1 || exit 1
run legacy || exit 1
