# Round 4: non-temporal store knob A/B at the final build (DTF_STORE_NT: bit 0 conv, 1 GEMM, 2 BN;
# default = 4, BN passes only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py > gpurun_out/r4_nt_$tag.json 2> gpurun_out/r4_nt_$tag.err || return 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r4_nt_$tag.json').read().strip().splitlines()[-1]); print(json.dumps({'tag': '$tag', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/r4_nt_ab.jsonl
}
run base0 DTF_X=0 || exit 1
run nt5 DTF_STORE_NT=5 || exit 1
run nt6 DTF_STORE_NT=6 || exit 1
run base1 DTF_X=0 || exit 1
run nt7 DTF_STORE_NT=7 || exit 1
run nt5b DTF_STORE_NT=5 || exit 1
run base2 DTF_X=0 || exit 1
