# Round 4: halo BNB with the x rows prefetched before the main loop: numerics, timings, ResNet A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py -k "halo_dgrad or bn_backward_sums or teacher" > gpurun_out/r4_t34.log 2>&1 || exit 1
timeout -k 10 180 python tools/halo_bnb_bench.py > gpurun_out/r4_halo_bnb_bench2.jsonl 2> gpurun_out/r4_halo_bnb_bench2.err || exit 1
for v in 1 0 1 0 1 0; do
  DTF_FUSE_BN_BWD_HALO=$v timeout -k 10 200 python bench.py > gpurun_out/r4_hb2_$v.json 2> gpurun_out/r4_hb2_$v.err || exit 1
  cat gpurun_out/r4_hb2_$v.json >> gpurun_out/r4_halo_bnb2_ab.jsonl
done
