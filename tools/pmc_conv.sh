#!/bin/bash
# PMC counters (own run: --pmc with kernel records only, no sys/runtime trace) for selected
# ResNet-50 conv shapes; keeps only the counter CSV + a per-kernel summary.
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
OUT="$R/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp || exit 1
LAYERS="${LAYERS:-s1b1c2,s2b1c1,s0b0c3}"
PMC="${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES}"
timeout -s KILL 180 rocprofv3 --pmc $PMC --output-format csv -d /tmp/pmc -o run -- \
  python3 "$R/tools/conv_bench.py" --only "$LAYERS" --iters 3 > "$OUT/run.log" 2>&1
rc=$?
find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} "$OUT/" \;
python3 "$R/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
exit $rc
