#!/bin/bash
# rocprofv3 kernel-trace + stats of the dtf ResNet-50 step and the stock-PyTorch comparator.
# Only the small *_stats.csv summaries are kept (full traces exceed gpurun's copy-back limit).
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT="$R/gpurun_out"
mkdir -p "$OUT"
cd /tmp || exit 1
prof() {  # name, args...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/prof_$name" -o run -- \
    python3 "$R/bench.py" "$@" > "$OUT/prof_$name.log" 2>&1
  local rc=$?
  mkdir -p "$OUT/prof_$name"
  find "/tmp/prof_$name" -name "*stats*.csv" -exec cp {} "$OUT/prof_$name/" \;
  python3 "$R/tools/summarize_trace.py" "/tmp/prof_$name" > "$OUT/prof_$name/summary.txt" 2>&1
  rm -rf "/tmp/prof_$name"
  return $rc
}
prof "${PROF_NAME:-dtf}" --steps 5 --warmup 3 ${DTF_BENCH_ARGS} || exit $?
[ -n "$SKIP_TORCH" ] || prof torch --impl torch --steps 5 --warmup 3
