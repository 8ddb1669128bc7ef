"""Cluster description, rendezvous and per-task servers (TF1 ``tf.train.Server`` semantics)."""
from .resolver import SimpleClusterResolver, TFConfigClusterResolver, export_torch_env
from .server import Server
from .spec import ClusterSpec, Config, from_flags, from_tf_config, split_host_port

__all__ = ["SimpleClusterResolver", "TFConfigClusterResolver", "export_torch_env", "Server",
           "ClusterSpec", "Config", "from_flags", "from_tf_config", "split_host_port"]
