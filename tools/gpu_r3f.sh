cd $GRAFT_REPO_ROOT && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3f &&
timeout -k 10 300 python -u -m pytest tests/test_gemm_pp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3f/pytest.log 2>&1 &&
timeout -k 10 400 python tools/gemm_bench.py --variants 8,11 --iters 20 --out gpurun_out/r3f/gemm_pp_vs_pingpong.jsonl > gpurun_out/r3f/gemm_bench.log 2>&1
