#!/bin/bash
# Kernel summaries of the ResNet-50 b1984 step with the tuned BN sweep grids and with the round-2
# grids (DTF_BN_GRID_CAP=2048 DTF_BN_STATS_BLOCKS=1024), same box.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
SKIP_TORCH=1 PROF_NAME=bn_new bash tools/prof_bench.sh || exit $?
DTF_BN_GRID_CAP=2048 DTF_BN_STATS_BLOCKS=1024 SKIP_TORCH=1 PROF_NAME=bn_old bash tools/prof_bench.sh || exit $?
