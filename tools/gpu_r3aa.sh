#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export PYTHONPATH=$PWD && mkdir -p gpurun_out/r3aa
timeout -k 10 300 python -u tools/stream_probe.py > gpurun_out/r3aa/probe.log 2>&1 || { tail -30 gpurun_out/r3aa/probe.log; exit 1; }
timeout -k 10 300 python -u tools/stream_probe.py --M 97216 --N 4096 > gpurun_out/r3aa/probe_n4096.log 2>&1 || { tail -30 gpurun_out/r3aa/probe_n4096.log; exit 1; }
