#!/bin/bash
# BERT: native dW for the small dense layers -- tests + A/B bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3w
timeout -k 10 300 python -u -m pytest tests/test_nlp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w/pytest_nlp.log 2>&1 || { tail -40 gpurun_out/r3w/pytest_nlp.log; exit 1; }
tail -2 gpurun_out/r3w/pytest_nlp.log
for i in 1 2; do
  DTF_DENSE_WGRAD_NATIVE=0 timeout -k 10 300 python -u bench.py --model bert_base --steps 20 --warmup 5 > gpurun_out/r3w/bert_off_$i.log 2>&1 || { tail -20 gpurun_out/r3w/bert_off_$i.log; exit 1; }
  timeout -k 10 300 python -u bench.py --model bert_base --steps 20 --warmup 5 > gpurun_out/r3w/bert_on_$i.log 2>&1 || { tail -20 gpurun_out/r3w/bert_on_$i.log; exit 1; }
done
