"""Multi-process data parallelism through the native GPU path: two ranks share the one MI355X of
the test box over gloo (RCCL refuses two ranks on one device), so the bucketed all-reduce meets
the HIP kernels' direct flat-buffer gradient writes exactly as in an 8-GPU run."""
import os
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)

pytestmark = pytest.mark.gpu


def test_two_rank_resnet50_allreduced_grads_equal_sum_of_local_grads(tmp_path):
    from distributedtensorflow_amd.cluster.launcher import free_ports
    import dist_worker
    port = free_ports(1)[0]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT,
                   OMP_NUM_THREADS="2")
        log = open(tmp_path / f"rank{r}.log", "w")
        procs.append((subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"),
                                        "resnet_gpu", str(tmp_path)], env=env, stdout=log,
                                       stderr=subprocess.STDOUT), log))
    try:
        for p, _ in procs:
            p.wait(timeout=100)
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
            log.close()
    for r, (p, _) in enumerate(procs):
        assert p.returncode == 0, open(tmp_path / f"rank{r}.log").read()[-3000:]
    res = [torch.load(tmp_path / f"rank{r}.pt") for r in range(2)]
    assert torch.equal(res[0]["grad"], res[1]["grad"])
    for k in res[0]["init"]:
        assert torch.equal(res[0]["init"][k], res[1]["init"][k]), k

    # reference: the same two half-batches through the same kernels in this process, summed
    from distributedtensorflow_amd import ops
    from distributedtensorflow_amd.models import resnet50
    from distributedtensorflow_amd.optimizers import MomentumOptimizer
    from distributedtensorflow_amd.parallel import OneDeviceStrategy
    x, y = dist_worker.resnet_batch()
    total = None
    for r in range(2):
        model = resnet50().cuda()
        model.load_state_dict(res[0]["init"])
        with OneDeviceStrategy("cuda").scope():
            opt = MomentumOptimizer(0.1, 0.9)
            loss = ops.sparse_softmax_cross_entropy(
                model(x[2 * r:2 * r + 2].cuda()), y[2 * r:2 * r + 2].cuda())
            opt.compute_gradients(loss, list(model.parameters()))
            torch.cuda.synchronize()
            g = opt.space.grad.cpu().clone()
        total = g if total is None else total + g
    assert torch.equal(res[0]["grad"], total)
    assert total.abs().sum() > 0
