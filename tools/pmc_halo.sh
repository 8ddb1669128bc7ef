#!/bin/bash
# 3x3 halo data gradients with fused BN-backward sums (conv.hip conv3x3_halo_kernel BNB): PMC
# counters in their own run (kernel records only), next to tools/halo_bnb_bench.py's timings.
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
OUT="$R/gpurun_out/pmc_halo"
mkdir -p "$OUT"
cd /tmp || exit 1
PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d /tmp/pmc_halo -o run -- \
  python3 "$R/tools/halo_bnb_bench.py" --iters 2 > "$OUT/run.log" 2>&1
rc=$?
find /tmp/pmc_halo -name "*counter_collection*.csv" -exec cp {} "$OUT/" \;
python3 "$R/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
exit $rc
