# Round 4: attention forward occupancy (step 20), then the conv roofline + ordered trace (step 16).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4_step20.sh || exit 1
bash tools/gpu_r4_step16.sh
