#!/bin/bash
# row-streaming GEMM timing probes: dbg 1 no C stores, 2 no MFMAs, 4 no A loads, 8 no B loads
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3q
timeout -k 10 300 python -u tools/gemm_bench.py --shapes 388864x1024x256,1555456x512x128,6221824x256x64 --variants 13 --dbg 0,1,2,3,4,8,12,15,0 --iters 10 --out gpurun_out/r3q/stream_probe.jsonl > gpurun_out/r3q/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3q/gemm_bench.log; exit 1; }
