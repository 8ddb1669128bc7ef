# Round 4: BN sums in the stride-2 3x3 dgrad epilogue only where the dgrad keeps its kernel
# (s1b0c2: 128 outputs, register implicit-GEMM either way): alternating A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_resnet_gpu.py -k "bn_backward_sums or teacher" > gpurun_out/r4_t41.log 2>&1 || exit 1
for v in 1 0 1 0 1 0; do
  DTF_FUSE_BN_BWD_S2=$v timeout -k 10 200 python bench.py > gpurun_out/r4_s2c_$v.json 2> gpurun_out/r4_s2c_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r4_s2c_$v.json').read().strip().splitlines()[-1]); print(json.dumps({'s2_bn_sums_c128': $v, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/r4_s2c_ab.jsonl
done
