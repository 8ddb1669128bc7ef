cd $GRAFT_REPO_ROOT && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3e &&
timeout -k 10 900 python bench.py --impl torch --batch 1984 --steps 10 --warmup 15 > gpurun_out/r3e/bench_torch_b1984.log 2>&1 ;
echo "rc=$?" >> gpurun_out/r3e/bench_torch_b1984.log
