"""Model zoo: the reference's MNIST CNN/MLP plus the north-star ResNet-50 and BERT-base."""
from .layers import (BatchNormalization, Conv2D, Dense, Layer, MaxPooling2D, NameScope,
                     collect_variables, name_scope)
from .mnist import MnistCNN, MnistMLP
from .resnet import ResNet, num_params, resnet50, resnet101, resnet152

__all__ = [
    "BatchNormalization", "Conv2D", "Dense", "Layer", "MaxPooling2D", "NameScope",
    "collect_variables", "name_scope", "MnistCNN", "MnistMLP", "ResNet", "num_params",
    "resnet50", "resnet101", "resnet152",
]
