# Round 4: BN sums in the stride-2 3x3 dgrad epilogues (DTF_FUSE_BN_BWD_S2) -- a longer
# alternating A/B, then a kernel profile with it on (bn_reduce per step).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 1 0 1 0 1 0 1 0; do
  DTF_FUSE_BN_BWD_S2=$v timeout -k 10 200 python bench.py > gpurun_out/r4_s2_$v.json 2> gpurun_out/r4_s2_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r4_s2_$v.json').read().strip().splitlines()[-1]); print(json.dumps({'s2_bn_sums': $v, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/r4_s2_ab.jsonl
done
DTF_FUSE_BN_BWD_S2=1 PROF_NAME=r4_resnet_s2 SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh
