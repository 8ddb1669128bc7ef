#!/bin/bash
# kernel profiles with the streamed-dgrad BN-backward fusion on and off
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD
SKIP_TORCH=1 PROF_NAME=r3y_bnb_on bash tools/prof_bench.sh || exit $?
DTF_FUSE_BN_BWD_STREAM=0 SKIP_TORCH=1 PROF_NAME=r3y_bnb_off bash tools/prof_bench.sh || exit $?
