cd $GRAFT_REPO_ROOT && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3c &&
timeout -k 10 300 python -u -m pytest tests/test_ps_dataplane.py -x -v -m gpu --timeout 60 --timeout-method thread > gpurun_out/r3c/pytest.log 2>&1
