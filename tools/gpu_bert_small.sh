#!/bin/bash
# BERT-side kernel changes: NLP + column-sum GPU tests, attention timing, BERT bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nlp.py tests/test_kernels_gpu.py -m gpu -k "attention or col_sum or bert or dense or nlp" > gpurun_out/bsm_tests.log 2>&1 || { tail -40 gpurun_out/bsm_tests.log; exit 1; }
tail -2 gpurun_out/bsm_tests.log
timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/bsm_attn.jsonl 2>/dev/null || exit 1
cat gpurun_out/bsm_attn.jsonl
for i in 1 2; do
timeout -k 10 300 python -u bench.py --model bert_base --steps 20 --warmup 5 > gpurun_out/bsm_bert_$i.log 2>&1 || exit 1
grep '^{' gpurun_out/bsm_bert_$i.log | cut -c1-160
done
