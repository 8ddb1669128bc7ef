"""train.py CLI end to end on CPU: OneDevice (BASELINE config 1), Mirrored over 2 gloo ranks under
torch.distributed.run, a between-graph PS cluster from config.json, checkpoint + restart."""
import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAIN = os.path.join(ROOT, "train.py")


@pytest.fixture(scope="module")
def data_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("mnist_cli")
    from distributedtensorflow_amd.data import mnist
    mnist.load_arrays(str(d), "train")
    mnist.load_arrays(str(d), "test")
    return str(d)


def _env():
    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TF_CONFIG"):
        e.pop(k, None)
    return e


def _result(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-3000:]
    return json.loads(lines[-1])


def test_onedevice_mlp_cpu(tmp_path, data_dir):
    r = subprocess.run([sys.executable, TRAIN, "--model", "mnist_mlp", "--strategy", "onedevice",
                        "--device", "cpu", "--max_steps", "60", "--log_every", "20",
                        "--data_dir", data_dir, "--log_dir", str(tmp_path / "tb"), "--eval"],
                       capture_output=True, text=True, env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = _result(r.stdout)
    assert res["global_step"] == 60 and res["test_accuracy"] > 0.5
    assert "Worker (0): loss = " in r.stdout
    assert glob.glob(str(tmp_path / "tb" / "*" / "events.out.tfevents.*"))


def test_checkpoint_and_restart(tmp_path, data_dir):
    ck = str(tmp_path / "ck")
    base = [sys.executable, TRAIN, "--model", "mnist_cnn", "--device", "cpu", "--strategy",
            "onedevice", "--data_dir", data_dir, "--log_dir", "", "--checkpoint_dir", ck,
            "--save_checkpoint_steps", "5", "--batch_size", "32"]
    r1 = subprocess.run(base + ["--max_steps", "10"], capture_output=True, text=True,
                        env=_env(), timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r2 = subprocess.run(base + ["--max_steps", "15"], capture_output=True, text=True,
                        env=_env(), timeout=300)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert "global step: 11)" in r2.stdout and "global step: 1)" not in r2.stdout
    assert _result(r2.stdout)["global_step"] == 15


def test_mirrored_two_ranks_torchrun(tmp_path, data_dir):
    from distributedtensorflow_amd.cluster.launcher import free_ports
    port = free_ports(1)[0]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={port}",
                        TRAIN, "--model", "mnist_cnn", "--strategy", "mirrored", "--device", "cpu",
                        "--max_steps", "6", "--batch_size", "16", "--data_dir", data_dir,
                        "--log_dir", ""], capture_output=True, text=True, env=_env(),
                       timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    res = _result(r.stdout)
    assert res["replicas"] == 2 and res["global_step"] == 6


def test_between_graph_cluster(tmp_path, data_dir):
    from distributedtensorflow_amd.cluster.launcher import launch_local
    codes, logs = launch_local(TRAIN, 1, 2, str(tmp_path),
                               ["--model=mnist_cnn", "--max_steps=12", "--batch_size=32",
                                f"--data_dir={data_dir}", "--log_dir=", "--device=cpu"],
                               env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2"}, timeout_s=300)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-2000:] for k, t in text.items()}
    assert "Close Parameter Server" in text["ps0"]
    assert _result(text["worker0"])["global_step"] >= 12


def _ports_args(n=3):
    from distributedtensorflow_amd.cluster.launcher import free_ports
    p = free_ports(n)
    return [f"--ps_hosts=127.0.0.1:{p[0]}",
            "--worker_hosts=" + ",".join(f"127.0.0.1:{x}" for x in p[1:])]


def test_template_mnist_replica_sync(tmp_path, data_dir):
    from distributedtensorflow_amd.cluster.launcher import launch_local
    codes, logs = launch_local(os.path.join(ROOT, "templates", "mnist_replica.py"), 1, 2,
                               str(tmp_path), _ports_args() + ["--train_steps=15",
                                                               f"--data_dir={data_dir}",
                                                               "--sync_replicas"],
                               env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2"}, timeout_s=300)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-2000:] for k, t in text.items()}
    for w in ("worker0", "worker1"):
        assert "validation cross entropy" in text[w] and "Training elapsed time" in text[w]


def test_template_between_graph_async_checkpoints(tmp_path, data_dir):
    from distributedtensorflow_amd.cluster.launcher import launch_local
    ck = str(tmp_path / "train_logs")
    codes, logs = launch_local(os.path.join(ROOT, "templates", "between_graph_async_mnist.py"),
                               1, 2, str(tmp_path), _ports_args() + [
                                   "--train_steps=25", f"--data_dir={data_dir}",
                                   f"--checkpoint_dir={ck}"],
                               env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2"}, timeout_s=300)
    text = {k: open(v).read() for k, v in logs.items()}
    assert all(c == 0 for c in codes.values()), {k: t[-2000:] for k, t in text.items()}
    from distributedtensorflow_amd.train import latest_checkpoint, load_variable
    ckpt = latest_checkpoint(ck)
    assert ckpt is not None
    assert int(load_variable(ckpt, "global_step")) >= 25
    assert load_variable(ckpt, "hid_w/Adagrad").shape == (784, 100)
