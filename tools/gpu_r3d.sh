cd $GRAFT_REPO_ROOT && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3d &&
timeout -k 10 400 python -u -m pytest tests/test_ps_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r3d/pytest_ps.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3d/bench_mirrored.log 2>&1 &&
timeout -k 10 300 python bench.py --strategy ps_async --num-workers 1 --steps 20 --warmup 5 --timeout 280 > gpurun_out/r3d/bench_ps_async1.log 2>&1 &&
timeout -k 10 400 python bench.py --strategy ps_async --num-workers 2 --steps 20 --warmup 5 --timeout 380 > gpurun_out/r3d/bench_ps_async2.log 2>&1
