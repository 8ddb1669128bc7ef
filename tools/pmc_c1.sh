#!/bin/bash
# Fused c3 backward kernels (conv1x1_bwd.hip) at the ResNet-50 b1984 shapes: PMC counters in their
# own run (kernel records only), next to tools/c1_bench.py's timings.
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
OUT="$R/gpurun_out/pmc_c1"
mkdir -p "$OUT"
cd /tmp || exit 1
PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d /tmp/pmc_c1 -o run -- \
  python3 "$R/tools/c1_bench.py" --iters 2 > "$OUT/run.log" 2>&1
rc=$?
find /tmp/pmc_c1 -name "*counter_collection*.csv" -exec cp {} "$OUT/" \;
python3 "$R/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
exit $rc
