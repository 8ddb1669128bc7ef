# Round 4: ResNet-50 b1984 knob A/B at the current build: stride-2 dgrad BN sums
# (DTF_FUSE_BN_BWD_S2), halo filter-in-registers (DTF_CONV_HALO_FREG), BN sums in every dgrad
# epilogue (DTF_FUSE_BN_BWD).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py > gpurun_out/r4_knob_$tag.json 2> gpurun_out/r4_knob_$tag.err || return 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r4_knob_$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/r4_knob_ab.jsonl
}
run base0 DTF_X=0 || exit 1
run s2 DTF_FUSE_BN_BWD_S2=1 || exit 1
run freg DTF_CONV_HALO_FREG=3 || exit 1
run base1 DTF_X=0 || exit 1
run bnball DTF_FUSE_BN_BWD=1 || exit 1
run s2b DTF_FUSE_BN_BWD_S2=1 || exit 1
run base2 DTF_X=0 || exit 1
