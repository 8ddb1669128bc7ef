# Round 4: steps 31 (halo BN-sum timings + PMC) and 32 (non-temporal store knob A/B).
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4_step31.sh || exit 1
bash tools/gpu_r4_step32.sh
