# Round 4: knob A/B (step 19), then the ResNet-50 v5 kernel profile (halo-epilogue BN1 sums in).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4_step19.sh || exit 1
PROF_NAME=r4_resnet_v5 SKIP_TORCH=1 DTF_BENCH_ARGS="" bash tools/prof_bench.sh
