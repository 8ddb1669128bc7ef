#!/bin/bash
# Same-box A/B of two builds of the HIP extension: arm A = the .so under ab/<name>/ (built from
# another tree state, e.g. `git stash; build; cp _lib/_dtf_hip*.so ab/<name>/; git stash pop;
# build`), arm B = the in-tree .so.  Runs `bench.py ARGS` alternately A B A B ... ROUNDS times,
# each under its own time limit, and prints one JSON line per run.
#   gpurun -- bash tools/ab_so.sh <name> <rounds> [bench.py args]
# AB_TOOL=tools/<probe>.py runs that probe (its JSON lines) in each arm instead of bench.py.
R="${GRAFT_REPO_ROOT:-/root/repo}"
NAME=${1:?name}; ROUNDS=${2:-2}; shift 2
TOOL=${AB_TOOL:-bench.py}
if [ "$TOOL" = bench.py ]; then ARGS=${*:-"--steps 20 --warmup 5"}; else ARGS=$*; fi
OUT="$R/gpurun_out/ab_$NAME"
mkdir -p "$OUT"
A=/tmp/ab_arm_a
rm -rf "$A" && mkdir -p "$A" && cp -r "$R/bench.py" "$R/distributedtensorflow_amd" "$R/tools" "$A/" || exit 1
cp "$R/ab/$NAME/"_dtf_hip*.so "$A/distributedtensorflow_amd/_lib/" || exit 1
for i in $(seq 1 "$ROUNDS"); do
  for arm in A B; do
    dir=$([ $arm = A ] && echo "$A" || echo "$R")
    ( cd "$dir" && PYTHONPATH="$dir" timeout -k 10 300 python -u $TOOL $ARGS ) \
      > "$OUT/${i}_$arm.log" 2>&1 || { tail -20 "$OUT/${i}_$arm.log"; exit 1; }
    if [ "$TOOL" = bench.py ]; then
      echo "{\"arm\": \"$arm\", \"round\": $i, \"bench\": $(grep '^{' "$OUT/${i}_$arm.log" | tail -1)}"
    else
      grep '^{' "$OUT/${i}_$arm.log" | sed "s/^{/{\"arm\": \"$arm\", \"round\": $i, /"
    fi
  done
done | tee "$OUT/ab.jsonl"
