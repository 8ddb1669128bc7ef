"""Distribution strategies and communication (RCCL over xGMI, one process per GPU)."""
from .health import (Heartbeat, HeartbeatHook, ReplicaConsistencyHook, ReplicaDivergence,
                     check_replicas_consistent, fingerprint)
from .ps_service import PSClient, ParameterServerService, assign_shards
from .ps_strategy import CentralStorageStrategy, ParameterServerStrategy
from .strategy import (BucketedAllReduce, MirroredStrategy, MultiWorkerMirroredStrategy,
                       OneDeviceStrategy, ReduceOp, Strategy, get_strategy, has_strategy,
                       init_process_group_from_env, verify_bucket_agreement)

__all__ = ["Heartbeat", "HeartbeatHook", "ReplicaConsistencyHook", "ReplicaDivergence",
           "check_replicas_consistent", "fingerprint", "PSClient", "ParameterServerService", "assign_shards", "CentralStorageStrategy",
           "ParameterServerStrategy", "BucketedAllReduce", "MirroredStrategy",
           "MultiWorkerMirroredStrategy", "OneDeviceStrategy", "ReduceOp", "Strategy",
           "get_strategy", "has_strategy", "init_process_group_from_env",
           "verify_bucket_agreement"]
