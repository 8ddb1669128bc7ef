# Round 4: BN1 backward sums from the 3x3 halo data-gradient epilogue: numerics, ResNet A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py -k "halo_dgrad or bn_backward_sums or direct_grad or lazy or teacher" > gpurun_out/r4_t17.log 2>&1 || exit 1
for v in 1 0 1 0; do
  DTF_FUSE_BN_BWD_HALO=$v timeout -k 10 200 python bench.py > gpurun_out/r4_bench_halobnb_$v.json 2> gpurun_out/r4_bench_halobnb_$v.err || exit 1
  cat gpurun_out/r4_bench_halobnb_$v.json >> gpurun_out/r4_halo_bnb_ab.jsonl
done
