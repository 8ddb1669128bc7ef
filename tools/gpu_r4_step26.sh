# Round 4: attention dropout keep bits stored by the forward for the fused backward: numerics,
# kernel timings, BERT-base A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nlp.py -k "attention or bert" > gpurun_out/r4_t26.log 2>&1 || exit 1
timeout -k 10 120 python tools/attn_bench.py > gpurun_out/r4_attn_keep.jsonl 2> gpurun_out/r4_attn_keep.err || exit 1
for v in 1 0 1 0; do
  DTF_ATTN_KEEP=$v timeout -k 10 240 python bench.py --model bert_base > gpurun_out/r4_bert_keep_$v.json 2> gpurun_out/r4_bert_keep_$v.err || exit 1
  cat gpurun_out/r4_bert_keep_$v.json >> gpurun_out/r4_bert_keep_ab.jsonl
done
