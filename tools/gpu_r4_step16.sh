# Round 4: per-shape conv roofline at b1984 (current kernels) + an ordered kernel trace of one
# ResNet-50 b1984 step (layer mapping for the weak 3x3 shapes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 600 python -u tools/conv_bench.py --batch 1984 --iters 5 > gpurun_out/r4_conv_roofline_b1984.jsonl 2> gpurun_out/r4_conv_roofline.err || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr16 -o run -- python3 $R/bench.py --steps 1 --warmup 2 > $R/gpurun_out/r4_trace16.log 2>&1 || exit 1
python3 $R/tools/trace_dump.py /tmp/tr16 --last 1200 > $R/gpurun_out/r4_resnet_step_trace.txt
