"""Cluster description (``config.json`` / flags / TF_CONFIG, reference
``run_mnist_distributed.py:14-43``) and the key/value logger (reference ``logger.py``)."""
import io
import json
import os

import pytest

from distributedtensorflow_amd.cluster import ClusterSpec, Config
from distributedtensorflow_amd.cluster.resolver import (SimpleClusterResolver,
                                                        TFConfigClusterResolver, export_torch_env)
from distributedtensorflow_amd.cluster.spec import from_flags, from_tf_config, split_host_port
from distributedtensorflow_amd.summary import logger


# ----------------------------------------------------------------------------- cluster
def test_config_json_order_and_hosts(tmp_path):
    p = tmp_path / "config.json"
    # JSON insertion order defines task order (not the numeric suffix)
    p.write_text('{"ps": {"ps:0": "h0:8001"}, '
                 '"workers": {"worker:1": "h2:6002", "worker:0": "h1:6001"}}')
    c = Config(str(p))
    assert c.get_ps_and_worker_hosts() == (("h0:8001",), ("h2:6002", "h1:6001"))
    assert c.get_workers_with_addresses() == (("worker:1", "worker:0"), ("h2:6002", "h1:6001"))
    spec = c.cluster_spec()
    assert spec.task_address("worker", 0) == "h2:6002"


def test_config_missing_key_message(tmp_path):
    p = tmp_path / "config.json"
    p.write_text('{"ps": {"ps:0": "h0:1"}}')
    with pytest.raises(AttributeError, match='"workers" configuration key'):
        Config(str(p))


def test_repo_config_json():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ps, workers = Config(os.path.join(root, "config.json")).get_ps_and_worker_hosts()
    assert len(ps) == 1 and len(workers) == 2


def test_cluster_spec_rank_layout():
    spec = ClusterSpec({"ps": ["p0:1", "p1:2"], "worker": ["w0:3", "w1:4", "w2:5"],
                        "chief": ["c:6"]})
    assert spec.jobs == ["chief", "worker", "ps"]
    assert spec.world_size() == 6
    assert [spec.task_of(r) for r in range(6)] == [("chief", 0), ("worker", 0), ("worker", 1),
                                                   ("worker", 2), ("ps", 0), ("ps", 1)]
    assert all(spec.rank_of(*spec.task_of(r)) == r for r in range(6))
    assert spec.chief() == ("chief", 0)
    assert spec.rendezvous_address() == ("c", 6)
    with pytest.raises(ValueError):
        spec.rank_of("worker", 3)
    assert ClusterSpec({"worker": {"1": "b:2", "0": "a:1"}}).job_tasks("worker") == ["a:1", "b:2"]


def test_from_flags_and_split():
    spec = from_flags("p:1,q:2", "a:3,b:4")
    assert spec.job_tasks("ps") == ["p:1", "q:2"] and spec.chief() == ("worker", 0)
    assert split_host_port("grpc://10.0.0.1:2222") == ("10.0.0.1", 2222)
    with pytest.raises(ValueError):
        split_host_port("nohost")


def test_tf_config_resolver(monkeypatch):
    cfg = {"cluster": {"worker": ["127.0.0.1:7000", "127.0.0.1:7001", "10.0.0.2:7000"],
                       "ps": ["10.0.0.2:7100"]},
           "task": {"type": "worker", "index": 2}}
    spec, job, idx = from_tf_config(json.dumps(cfg))
    assert (job, idx) == ("worker", 2)
    r = TFConfigClusterResolver(cfg)
    assert r.rank == 2 and r.world_size == 4
    assert r.local_rank() == 0                      # first task on 10.0.0.2
    assert SimpleClusterResolver(spec, "ps", 0).local_rank() == 1
    for k in ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    env = export_torch_env(r)
    assert env == {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "7000", "WORLD_SIZE": "4",
                   "RANK": "2", "LOCAL_RANK": "0"}
    assert os.environ["RANK"] == "2"


# ----------------------------------------------------------------------------- logger
def test_human_format_table():
    buf = io.StringIO()
    f = logger.HumanOutputFormat(buf)
    f.writekvs({"b": 1.23456, "a": "x" * 40})
    lines = buf.getvalue().strip().split("\n")
    assert lines[0].startswith("---") and lines[-1].startswith("---")
    assert lines[1].startswith("| a ") and "..." in lines[1]   # sorted, clipped at 20 chars
    assert "1.23" in lines[2]
    with pytest.raises(TypeError):
        logger.HumanOutputFormat(42)


def test_configure_formats_and_readers(tmp_path, monkeypatch):
    monkeypatch.delenv("RANK", raising=False)
    d = str(tmp_path / "logs")
    with logger.scoped_configure(d, ["log", "json", "csv", "tensorboard"]):
        for i in range(3):
            logger.logkv("it", i)
            logger.logkv_mean("loss", 1.0)
            logger.logkv_mean("loss", 3.0)
            if i == 2:
                logger.logkv("late", 7)
            logger.dumpkvs()
        logger.info("hello", "world")
        logger.debug("hidden")
        assert logger.get_dir() == d
    assert os.path.exists(os.path.join(d, "log.txt"))
    txt = open(os.path.join(d, "log.txt")).read()
    assert "hello world" in txt and "hidden" not in txt
    js = logger.read_json(os.path.join(d, "progress.json"))
    assert list(js["it"]) == [0, 1, 2] and list(js["loss"]) == [2.0, 2.0, 2.0]
    csv = logger.read_csv(os.path.join(d, "progress.csv"))
    assert list(csv.columns) == ["it", "loss", "late"]     # header grew, rows padded
    assert csv["late"].isna().sum() == 2 and csv["late"].iloc[2] == 7
    tb = logger.read_tb(os.path.join(d, "tb"))
    assert list(tb["it"]) == [0.0, 1.0, 2.0]


def test_rank_suffix_and_profile(tmp_path, monkeypatch):
    monkeypatch.setenv("RANK", "3")
    monkeypatch.delenv("OPENAI_LOG_FORMAT_MPI", raising=False)
    d = str(tmp_path / "r3")
    with logger.scoped_configure(d):
        @logger.profile("work")
        def f():
            return 5
        assert f() == 5
        assert "wait_work" in logger.getkvs()
        logger.record_tabular("x", 1)
        logger.dump_tabular()
    assert os.path.exists(os.path.join(d, "log-rank003.txt"))


def test_tensorboard_writer_reference_signature(tmp_path):
    """``TensorBoardOutputFormat(dir).writekvs(kvs, global_step=n)`` as used by
    ``run_mnist_distributed.py:167``."""
    from distributedtensorflow_amd.summary.events import read_scalars
    tb = logger.TensorBoardOutputFormat(dir=str(tmp_path))
    tb.writekvs({"Global Step": 5, "Loss": 0.5}, global_step=5)
    tb.writekvs({"Global Step": 6, "Loss": 0.25}, global_step=6)
    tb.close()
    sc = read_scalars(str(tmp_path))
    assert sc["Loss"] == [(5, 0.5), (6, 0.25)]


def test_usable_cpus_clamps_thread_pools(monkeypatch):
    """ConfigProto(intra_op_parallelism_threads=os.cpu_count()) (the reference's setting) must
    not oversubscribe a CPU quota: threads are clamped to usable_cpus()."""
    import torch

    from distributedtensorflow_amd.train import ConfigProto
    from distributedtensorflow_amd.utils.cpu import usable_cpus
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    assert usable_cpus() <= 2
    prev = torch.get_num_threads()
    try:
        ConfigProto(intra_op_parallelism_threads=4096).apply()
        assert torch.get_num_threads() <= 2
    finally:
        torch.set_num_threads(prev)
