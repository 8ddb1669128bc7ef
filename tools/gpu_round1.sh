#!/bin/bash
# First GPU session: kernel numerics, smoke, comparator + framework bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" ; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "gpurun_out/$name.log"; echo "$name rc=$rc"
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }  # 1 = assertion failures, no GPU fault
python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/env.log 2>&1
run pytest_kernels 600 python -m pytest tests/test_kernels_gpu.py -q -rf ; r=$?; ok $r || exit $r
run smoke 300 python __graft_entry__.py smoke ; r=$?; ok $r || exit $r
run bench_torch 400 python bench.py --impl torch --steps 10 --warmup 5 ; r=$?; ok $r || exit $r
run bench_dtf 400 python bench.py --impl dtf --steps 10 --warmup 3 ; r=$?
exit $r
