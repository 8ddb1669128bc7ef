#!/bin/bash
# row-streaming GEMM skeleton probes (timing only): 15 = no stores/MFMA/A/B traffic; +16 no LDS
# staging, +32 no barrier, +64 no DMA instructions, +128 no B fragment reads
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u tools/gemm_bench.py --shapes 388864x1024x256,6221824x256x64 --variants 13 --dbg 0,15,31,47,79,143,255,16,128,64,0 --iters 10 --out gpurun_out/r3s/stream_probe.jsonl > gpurun_out/r3s/gemm_bench.log 2>&1 || { tail -30 gpurun_out/r3s/gemm_bench.log; exit 1; }
