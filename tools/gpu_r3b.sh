cd $GRAFT_REPO_ROOT && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3b &&
timeout -k 10 200 python tools/determinism_probe.py 32 128 > gpurun_out/r3b/determinism.log 2>&1
