#!/bin/bash
# Offline hipBLASLt solution tuning (PyTorch TunableOp) of the BERT bench GEMMs, then a same-box
# A/B of the tuned table against the default heuristics.  Writes gpurun_out/tuning/.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
OUT=gpurun_out/tuning
mkdir -p "$OUT" distributedtensorflow_amd/tuning
MODEL=${MODEL:-bert_base}
PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 ${TUNE_TIMEOUT:-900} python -u bench.py --model $MODEL \
  --steps 1 --warmup 1 --gemm-tuning tune --gemm-tuning-out "$OUT/tunableop_$MODEL.csv" \
  > "$OUT/tune.log" 2>&1 || exit $?
cp "$OUT/tunableop_$MODEL.csv" distributedtensorflow_amd/tuning/ || exit 1
for m in off auto off auto; do
  timeout -k 10 300 python -u bench.py --model $MODEL --steps 20 --warmup 5 --gemm-tuning $m \
    > "$OUT/bench_$m.log" 2>&1 || exit $?
  echo "$m $(tail -1 "$OUT/bench_$m.log" | cut -c1-160)" >> "$OUT/summary.txt"
done
