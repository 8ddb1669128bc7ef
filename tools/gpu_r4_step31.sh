# Round 4: halo-epilogue BN sums -- timings (fused vs reduce pass) and PMC counters of the halo
# kernels with and without the BNB epilogue.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 180 python tools/halo_bnb_bench.py > gpurun_out/r4_halo_bnb_bench.jsonl 2> gpurun_out/r4_halo_bnb_bench.err || exit 1
bash tools/pmc_halo.sh
