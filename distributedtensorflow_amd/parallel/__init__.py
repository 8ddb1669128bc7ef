"""Distribution strategies and communication (RCCL over xGMI, one process per GPU)."""
from .strategy import (BucketedAllReduce, MirroredStrategy, MultiWorkerMirroredStrategy,
                       OneDeviceStrategy, ReduceOp, Strategy, get_strategy, has_strategy,
                       init_process_group_from_env)

__all__ = ["BucketedAllReduce", "MirroredStrategy", "MultiWorkerMirroredStrategy",
           "OneDeviceStrategy", "ReduceOp", "Strategy", "get_strategy", "has_strategy",
           "init_process_group_from_env"]
