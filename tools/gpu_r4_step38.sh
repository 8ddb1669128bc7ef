# Round 4: confirm the BN reduce-pass block target 512 (DTF_BN_STATS_BLOCKS) against the default
# 1024, alternating on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 512 1024 512 1024 512 1024; do
  DTF_BN_STATS_BLOCKS=$v timeout -k 10 200 python bench.py > gpurun_out/r4_sb_$v.json 2> gpurun_out/r4_sb_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r4_sb_$v.json').read().strip().splitlines()[-1]); print(json.dumps({'stats_blocks': $v, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/r4_stats_blocks_ab.jsonl
done
