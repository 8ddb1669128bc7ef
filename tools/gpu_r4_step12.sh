# Round 4: 16-B half-wave LayerNorm kernels: numerics + BERT A/B (DTF_LN_WIDE 1 = forward only,
# 3 = forward + backward, 0 = the 8-B kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nlp.py > gpurun_out/r4_t12.log 2>&1 || exit 1
for m in 1 0 3 1; do
  DTF_LN_WIDE=$m timeout -k 10 200 python bench.py --model bert_base > gpurun_out/r4_bench_ln$m.json 2> gpurun_out/r4_bench_ln$m.err || exit 1
  cp gpurun_out/r4_bench_ln$m.json gpurun_out/r4_bench_ln${m}_$(date +%s).json
done
