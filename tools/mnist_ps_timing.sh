#!/bin/bash
# The reference's own workload (run_mnist_distributed.py: MNIST CNN, batch 128, Adam 5e-4, async
# PS, 1000 global steps) timed end to end on the GPU box (EXTRA="--dtype fp32" = reference precision).  PLANES: ipc = PS shard in HBM, workers
# push/pull through hipIpc mappings (default); gloo = round-1 host path (PS on the CPU, tensors
# over TCP).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && export PYTHONPATH="$R" && mkdir -p gpurun_out/mnist_ps
for plane in ${PLANES:-ipc}; do
 if [ "$plane" = gloo ]; then PF="--ps_device cpu --data_plane gloo"; else PF="--ps_device gpu --data_plane auto"; fi
for nw in ${WORKERS:-1 2}; do
 for dev in ${DEVICES:-gpu}; do
  s=$(date +%s.%N)
  d=gpurun_out/mnist_ps/${plane}_w${nw}_$dev
  timeout -k 10 ${TMO:-300} python -m distributedtensorflow_amd.cluster.launcher run_mnist_distributed.py \
    --num_ps 1 --num_workers $nw --workdir $d --device $dev $PF ${EXTRA} > $d.json 2>&1 || exit $?
  e=$(date +%s.%N)
  t=$(grep "Training elapsed" $d/worker0.log | awk '{print $4}')
  ps=$(grep "Close Parameter Server" $d/ps0.log | sed "s/.*Server ... //" | tr "'" '"' | sed 's/False/false/;s/True/true/')
  echo "{\"workload\": \"reference run_mnist_distributed.py, 1 PS + $nw workers ($dev), ${STEPS_N:-1000} global steps\", \"data_plane\": \"$plane\", \"ps_stats\": ${ps:-null}, \"wall_s\": $(python -c "print(round($e-$s,2))"), \"train_s\": ${t:-null}}" | tee -a gpurun_out/mnist_ps/timing.jsonl
 done
done
done
