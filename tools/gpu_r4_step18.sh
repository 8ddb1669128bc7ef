# Round 4: step 17 (halo-epilogue BN1 sums: numerics + ResNet A/B), then step 16's conv roofline
# and ordered step trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4_step17.sh || exit 1
sed -i 's/--iters 10/--iters 5/' tools/gpu_r4_step16.sh
bash tools/gpu_r4_step16.sh
