#!/bin/bash
# PMC counters of the TN weight-gradient kernel on one dense shape (own runs, kernel records only).
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
OUT="$R/gpurun_out/pmc_wgrad"
mkdir -p "$OUT"
cd /tmp || exit 1
n=0
for PMC in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d /tmp/pmcw$n -o run -- \
    python3 "$R/tools/wgrad_one.py" ${SHAPE:-65536 2304 768} > "$OUT/run$n.log" 2>&1 || exit $?
  mkdir -p "$OUT/p$n"
  find /tmp/pmcw$n -name "*counter_collection*.csv" -exec cp {} "$OUT/p$n/" \;
  python3 "$R/tools/summarize_pmc.py" "$OUT/p$n" > "$OUT/summary$n.txt" 2>&1
done
