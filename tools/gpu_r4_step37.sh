# Round 4: last knob sweep at the final build (wgrad pipeline, small-K conv bits, BN reduce-pass
# block target, BN grid cap, GEMM-route threshold for 1x1 convs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py > gpurun_out/r4_k2_$tag.json 2> gpurun_out/r4_k2_$tag.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r4_k2_$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/r4_knob2_ab.jsonl
}
run base0 DTF_X=0 || exit 1
run pipe0 DTF_WGRAD_PIPE=0 || exit 1
run sk15 DTF_CONV_SMALL_K=15 || exit 1
run stats2048 DTF_BN_STATS_BLOCKS=2048 || exit 1
run base1 DTF_X=0 || exit 1
run stats512 DTF_BN_STATS_BLOCKS=512 || exit 1
run cap2048 DTF_BN_GRID_CAP=2048 || exit 1
run min256 DTF_GEMM_1X1_MIN_C=256 || exit 1
run base2 DTF_X=0 || exit 1
run min1024 DTF_GEMM_1X1_MIN_C=1024 || exit 1
run base3 DTF_X=0 || exit 1
