#!/bin/bash
# PMC counters of the hand-written GEMM (csrc/kernels/gemm.hip) next to hipBLASLt on one shape.
# Own run: --pmc with kernel records only (no sys/runtime trace).
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
OUT="$R/gpurun_out/pmc_gemm"
mkdir -p "$OUT"
cd /tmp || exit 1
PMC="${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES}"
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d /tmp/pmcg -o run -- \
  python3 "$R/tools/gemm_bench.py" --only "${SHAPES:-bert_ffn2_fwd}" --iters 3 --variants "${VARIANTS:-0}" > "$OUT/run.log" 2>&1
rc=$?
find /tmp/pmcg -name "*counter_collection*.csv" -exec cp {} "$OUT/" \;
python3 "$R/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
exit $rc
