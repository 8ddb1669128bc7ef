#!/bin/bash
# Attention kernel timing + PMC counters (own run, kernel records only) at the BERT-base shape
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
OUT="$R/gpurun_out/pmc_attn"
mkdir -p "$OUT"
timeout -k 10 120 python3 "$R/tools/attn_bench.py" > "$OUT/attn_bench.jsonl" 2> "$OUT/attn_bench.err" || exit $?
cd /tmp || exit 1
PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d /tmp/pmc -o run -- \
  python3 "$R/tools/attn_bench.py" --iters 2 > "$OUT/run.log" 2>&1
rc=$?
find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} "$OUT/" \;
python3 "$R/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
exit $rc
