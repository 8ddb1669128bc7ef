# Round 4: attention forward at 6 / 8 waves per SIMD (DTF_ATTN_FWD_OCC): kernel timings + errors,
# attention tests at 6, BERT-base A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for o in 0 6 8 0; do
  timeout -k 10 120 python tools/attn_bench.py --fwd-occ $o >> gpurun_out/r4_attn_occ.jsonl 2>> gpurun_out/r4_attn_occ.err || exit 1
done
DTF_ATTN_FWD_OCC=6 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nlp.py -k "attention" > gpurun_out/r4_t20.log 2>&1 || exit 1
for v in 6 0 6 0; do
  DTF_ATTN_FWD_OCC=$v timeout -k 10 240 python bench.py --model bert_base > gpurun_out/r4_bert_occ_$v.json 2> gpurun_out/r4_bert_occ_$v.err || exit 1
  cat gpurun_out/r4_bert_occ_$v.json >> gpurun_out/r4_bert_occ_ab.jsonl
done
