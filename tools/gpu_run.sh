#!/bin/bash
# One parameterised GPU runner (replaces the per-step tools/gpu_r3*.sh / gpu_r4_step*.sh scripts).
#
#   gpurun -- bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# STEP is one of
#   pytest:<pytest args>       e.g. "pytest:tests/test_ps_gpu.py -k killed"
#   gpu-suite                  every gpu-marked test (-x, verbose, per-test thread timeout)
#   smoke                      __graft_entry__.smoke()
#   bench:<bench.py args>      e.g. "bench:--steps 20 --warmup 5"
#   prof:<name>:<bench args>   rocprofv3 kernel trace + stats -> gpurun_out/prof_<name>/summary.txt
#   py:<script> [args]         any tools/ python probe
#   sh:<command>               a shell command line (env-var A/B arms: "sh:DTF_X=1 python bench.py")
#   env:<K=V>                  export K=V for every later step of this call (e.g. before a prof:);
#                              env:PYTEST_K=<expr> gives later pytest: steps a -k expression (spaces ok)
# Each step runs under its own time limit (STEP_TIMEOUT, default 600 s), logs to
# gpurun_out/<TAG>/<n>_<kind>.log, and the run stops at the first failing step (no retries):
# after a fault, abort, segfault or time limit nothing more touches the GPU in this call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}; shift
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONPATH="$R" TMPDIR=/tmp
T=${STEP_TIMEOUT:-600}
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  log="$OUT/${n}_${kind}.log"
  echo "[gpu_run] step $n: $step" | tee -a "$OUT/steps.txt"
  t0=$(date +%s)
  case "$kind" in
    pytest) if [ -n "$PYTEST_K" ]; then
              timeout -k 10 "$T" python -u -m pytest -x -v --timeout 200 --timeout-method thread -k "$PYTEST_K" $arg > "$log" 2>&1
            else
              timeout -k 10 "$T" python -u -m pytest -x -v --timeout 200 --timeout-method thread $arg > "$log" 2>&1
            fi ;;
    gpu-suite) timeout -k 10 "$T" python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=25 > "$log" 2>&1 ;;
    smoke) timeout -k 10 "$T" python -u __graft_entry__.py smoke > "$log" 2>&1 ;;
    bench) timeout -k 10 "$T" python -u bench.py $arg > "$log" 2>&1 ;;
    prof)
      name=${arg%%:*}; bargs=${arg#*:}; [ "$bargs" = "$arg" ] && bargs=""
      mkdir -p "$OUT/prof_$name"
      ( cd /tmp && timeout -k 10 "$T" rocprofv3 --kernel-trace --stats --output-format csv \
          -d "/tmp/prof_$name" -o run -- python3 "$R/bench.py" $bargs ) > "$log" 2>&1
      rc=$?
      find "/tmp/prof_$name" -name "*stats*.csv" -exec cp {} "$OUT/prof_$name/" \;
      python3 "$R/tools/summarize_trace.py" "/tmp/prof_$name" > "$OUT/prof_$name/summary.txt" 2>&1
      # the ordered dispatch list of the last ~1.3 steps (layer mapping: tools/trace_dump.py)
      python3 "$R/tools/trace_dump.py" "/tmp/prof_$name" --last ${TRACE_LAST:-900} --min-us 5 \
        > "$OUT/prof_$name/trace_tail.txt" 2>&1
      # GPU idle inside the last step (dispatches per step: GAP_LAST, ResNet-50 ~645, BERT ~816)
      python3 "$R/tools/trace_gaps.py" "/tmp/prof_$name" --last ${GAP_LAST:-645} \
        > "$OUT/prof_$name/gaps.txt" 2>&1
      rm -rf "/tmp/prof_$name"
      (exit $rc) ;;
    py) timeout -k 10 "$T" python -u $arg > "$log" 2>&1 ;;
    sh) timeout -k 10 "$T" bash -c "$arg" > "$log" 2>&1 ;;
    env) export "$arg"; echo "$arg" > "$log" ;;
    *) echo "unknown step kind: $kind" >&2; exit 2 ;;
  esac
  rc=$?
  echo "[gpu_run] step $n rc=$rc in $(( $(date +%s) - t0 )) s" | tee -a "$OUT/steps.txt"
  if [ $rc -ne 0 ]; then
    tail -60 "$log"
    exit $rc
  fi
  tail -3 "$log"
done
