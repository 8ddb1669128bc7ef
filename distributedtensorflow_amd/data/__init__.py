"""Input pipelines: tf.data-style Dataset, MNIST idx (offline synthetic fallback), synthetic
ImageNet / MLM generators for benchmarks."""
from . import mnist
from .dataset import Dataset, Iterator, NativeBatchDataset
from .device import DeviceArrayDataset
from .synthetic import SyntheticImageNet, SyntheticMLM

__all__ = ["mnist", "Dataset", "DeviceArrayDataset", "Iterator", "NativeBatchDataset",
           "SyntheticImageNet", "SyntheticMLM"]
