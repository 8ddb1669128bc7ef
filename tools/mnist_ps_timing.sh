#!/bin/bash
# The reference's own workload (run_mnist_distributed.py: MNIST CNN, batch 128, Adam 5e-4, async
# PS, 1000 global steps) timed end to end on the GPU box: PS on the CPU, workers on the GPU.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONPATH="$R" && mkdir -p gpurun_out/mnist_ps
for nw in ${WORKERS:-1 2}; do
 for dev in ${DEVICES:-gpu}; do
  s=$(date +%s.%N)
  d=gpurun_out/mnist_ps/w${nw}_$dev
  timeout -k 10 ${TMO:-300} python -m distributedtensorflow_amd.cluster.launcher run_mnist_distributed.py \
    --num_ps 1 --num_workers $nw --workdir $d --device $dev ${EXTRA} > $d.json 2>&1 || exit $?
  e=$(date +%s.%N)
  t=$(grep "Training elapsed" $d/worker0.log | awk '{print $4}')
  echo "{\"workload\": \"reference run_mnist_distributed.py, 1 PS + $nw workers ($dev), ${STEPS_N:-1000} global steps\", \"wall_s\": $(python -c "print(round($e-$s,2))"), \"train_s\": ${t:-null}}" | tee -a gpurun_out/mnist_ps/timing.jsonl
 done
done
