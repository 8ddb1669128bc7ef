cd $GRAFT_REPO_ROOT && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3a &&
timeout -k 10 900 python -u -m pytest tests/test_forced_reducer_gpu.py tests/test_bench_multirank_gpu.py tests/test_ps_dataplane.py tests/test_ps_gpu.py -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/r3a/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3a/bench.log 2>&1
