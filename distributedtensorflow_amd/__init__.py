"""distributedtensorflow_amd — an MI355X-native distributed training framework.

Capabilities of SvenGronauer/distributedTensorFlow (TF1 parameter-server / worker MNIST
training, logger, TensorBoard events, checkpoints) re-designed for AMD MI355X (gfx950):
PyTorch-ROCm tensors + hand-written HIP/CDNA4 kernels + RCCL over xGMI, one process per GPU,
with a tf.distribute-style strategy API.
"""
__version__ = "0.1.0"

from . import ops  # noqa: F401

__all__ = ["ops", "__version__"]
