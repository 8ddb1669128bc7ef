#!/bin/bash
# PMC counters of every kernel of a short bench.py run (default: the ResNet-50 b1984 step), two
# passes in their own runs (rocprofv3 --pmc only, no traces): SQ issue/wait breakdown + MFMA busy,
# then L2 traffic (FETCH_SIZE, WRITE_SIZE) + GRBM_GUI_ACTIVE (clock).  Summaries:
# gpurun_out/pmc_step/{sq,tcc}/summary.txt.  PMC_MEM_ONLY=1: one memory-pipe pass instead
# (gpurun_out/pmc_step/mem/summary.txt).  PMC_INST=1: one instruction-mix pass (VALU / LDS / MFMA
# instructions and active cycles per wave: which kernels are VALU-issue bound)
# (gpurun_out/pmc_step/inst/summary.txt).
#   gpurun -- bash tools/pmc_step.sh [bench.py args]
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export PYTHONPATH="$R${PYTHONPATH:+:$PYTHONPATH}"
ARGS=${*:-"--steps 2 --warmup 1"}
cd /tmp || exit 1
run_pass() {
  local name=$1; shift
  local out="$R/gpurun_out/pmc_step/$name"
  mkdir -p "$out"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "/tmp/pmc_$name" -o run -- \
    python3 "$R/bench.py" $ARGS > "$out/run.log" 2>&1
  local rc=$?
  find "/tmp/pmc_$name" -name "*counter_collection*.csv" -exec cp {} "$out/" \;
  python3 "$R/tools/summarize_pmc.py" "$out" > "$out/summary.txt" 2>&1
  rm -rf "/tmp/pmc_$name"
  return $rc
}
if [ -n "$PMC_MEM_ONLY" ]; then
  # memory-pipe pass only: address-unit busy / stalls behind the L2, vector L1 stall and request
  # latency (TA 2, TCP 4, GRBM 1 counters: one pass)
  run_pass mem TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES \
    TCP_TCR_TCP_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_WRITE_REQ_LATENCY GRBM_GUI_ACTIVE
  exit $?
fi
if [ -n "$PMC_INST" ]; then
  run_pass inst SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS
  exit $?
fi
run_pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES &&
run_pass tcc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT
