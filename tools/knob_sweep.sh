#!/bin/bash
# Same-box sweep of the kernel-variant switches at the bench default (ResNet-50 b2048): the
# baseline runs first and last (drift check).  One JSON line per run in gpurun_out/sweep/.
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/sweep"
mkdir -p "$OUT"
cd "$R" || exit 1
export PYTHONPATH="$R"
run() {  # label, env assignments...
  local label=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 15 --warmup 4 > "$OUT/$label.log" 2>&1 || return $?
  echo "$label $(tail -1 "$OUT/$label.log" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')" | tee -a "$OUT/summary.txt"
}
: > "$OUT/summary.txt"
run base DTF_NOP=1 || exit $?
DEFAULT_SWEEP="fuse_bn_bwd:DTF_FUSE_BN_BWD=1 conv_dma0:DTF_CONV_DMA=0 conv_dma1:DTF_CONV_DMA=1 wgrad_pipe1:DTF_WGRAD_PIPE=1 wgrad_pipe2:DTF_WGRAD_PIPE=2 small_k0:DTF_CONV_SMALL_K=0 conv_gemm0:DTF_CONV_GEMM=0 store_nt7:DTF_STORE_NT=7"
for spec in ${SWEEP:-$DEFAULT_SWEEP}; do
  run "${spec%%:*}" "${spec#*:}" || exit $?
done
run base2 DTF_NOP=1 || exit $?
