#!/bin/bash
# FFN data gradient with the GELU derivative in our GEMM's epilogue (DTF_BERT_FUSE_GELU_DGRAD=1)
# vs hipBLASLt dgrad + bias_gelu backward; tests first, then alternating same-box benches
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_nlp.py tests/test_dense_gpu.py tests/test_gemm_pp_gpu.py tests/test_kernels_gpu.py -m gpu -k "gelu or gemm or dense or bert or attention" > gpurun_out/gd_tests.log 2>&1 || { tail -40 gpurun_out/gd_tests.log; exit 1; }
tail -2 gpurun_out/gd_tests.log
for i in 1 2; do
  for f in 1 0; do
    DTF_BERT_FUSE_GELU_DGRAD=$f timeout -k 10 300 python -u bench.py --model bert_base --steps 20 --warmup 5 > gpurun_out/gd_${f}_$i.log 2>&1 || exit 1
    grep '^{' gpurun_out/gd_${f}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('fused', $f, d['value'], d['ms_per_step'], d['config'].get('final_loss'))"
  done
done
