# Round 4: PMC counters of the new kernels (fused c3 backward, fused attention backward) and
# kernel profiles of both benches at the round's final state.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/pmc_c1.sh || exit 1
bash tools/pmc_attn.sh || exit 1
PROF_NAME=r4_resnet_v4 SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh || exit 1
PROF_NAME=r4_bert_v2 SKIP_TORCH=1 DTF_BENCH_ARGS="--model bert_base" bash tools/prof_bench.sh
