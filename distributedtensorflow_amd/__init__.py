"""distributedtensorflow_amd — an MI355X-native distributed training framework.

Capabilities of SvenGronauer/distributedTensorFlow (TF1 parameter-server / worker MNIST
training, logger, TensorBoard events, checkpoints) re-designed for AMD MI355X (gfx950):
PyTorch-ROCm tensors + hand-written HIP/CDNA4 kernels + RCCL over xGMI, one process per GPU,
with a tf.distribute-style strategy API.

    import distributedtensorflow_amd as dtf
    strategy = dtf.distribute.MirroredStrategy()
    with strategy.scope():
        model = dtf.models.resnet50()
        opt = dtf.train.MomentumOptimizer(0.1, 0.9)
"""
__version__ = "0.1.0"

from . import cluster, data, models, ops, optimizers, parallel, profiler, summary, train  # noqa: F401
from . import parallel as distribute  # tf.distribute-style alias
from .summary import logger  # noqa: F401

# tf.train optimizer names live under train too
for _n in ("AdamOptimizer", "AdagradOptimizer", "MomentumOptimizer", "GradientDescentOptimizer",
           "SyncReplicasOptimizer", "LAMBOptimizer"):
    setattr(train, _n, getattr(optimizers, _n))
train.Server = cluster.Server
train.ClusterSpec = cluster.ClusterSpec

__all__ = ["cluster", "data", "models", "ops", "optimizers", "parallel", "distribute", "profiler",
           "summary", "train", "logger", "__version__"]
