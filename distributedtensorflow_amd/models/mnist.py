"""The reference's two MNIST models.

* :class:`MnistCNN` — ``create_model`` of ``run_mnist_distributed.py:46-70``: reshape to
  ``[-1,28,28,1]``, conv5x5x32 SAME+ReLU, maxpool 2/2, conv5x5x64 SAME+ReLU, maxpool 2/2,
  flatten 3136, dense 1024+ReLU, dense 10.  3,274,634 parameters, tf.layers names
  ``conv2d``, ``conv2d_1``, ``dense``, ``dense_1``.
* :class:`MnistMLP` — ``templates/00_mnist_replica.py:138-164``: 784 -> hidden (100) ReLU ->
  10; truncated-normal init (stddev 1/28 and 1/sqrt(hidden)), zero biases, variables
  ``hid_w, hid_b, sm_w, sm_b``.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2D, Dense, Layer, MaxPooling2D, _tag, name_scope, truncated_normal_

IMAGE_PIXELS = 28


class MnistCNN(Layer):
    input_signature_shape = (None, 784)      # SavedModel serving input (flat 28x28 images)

    def __init__(self, num_classes=10):
        super().__init__()
        with name_scope():
            self.conv1 = Conv2D(1, 32, 5, padding="same", activation="relu")
            self.pool1 = MaxPooling2D(2, 2)
            self.conv2 = Conv2D(32, 64, 5, padding="same", activation="relu")
            self.pool2 = MaxPooling2D(2, 2)
            self.dense = Dense(7 * 7 * 64, 1024, activation="relu")
            self.logits = Dense(1024, num_classes)

    def forward(self, x):
        x = x.reshape(-1, 28, 28, 1)
        y = self.pool1(self.conv1(x))
        y = self.pool2(self.conv2(y))
        y = y.reshape(y.shape[0], 7 * 7 * 64)
        y = self.dense(y)
        return self.logits(y).float()


class MnistMLP(Layer):
    input_signature_shape = (None, 784)

    def __init__(self, hidden_units=100, num_classes=10):
        super().__init__()
        self.hid_w = _tag(nn.Parameter(torch.empty(IMAGE_PIXELS * IMAGE_PIXELS, hidden_units)),
                          "hid_w")
        truncated_normal_(self.hid_w.data, 1.0 / IMAGE_PIXELS)
        self.hid_b = _tag(nn.Parameter(torch.zeros(hidden_units)), "hid_b")
        self.sm_w = _tag(nn.Parameter(torch.empty(hidden_units, num_classes)), "sm_w")
        truncated_normal_(self.sm_w.data, 1.0 / math.sqrt(hidden_units))
        self.sm_b = _tag(nn.Parameter(torch.zeros(num_classes)), "sm_b")

    def forward(self, x):
        """Returns logits; the template applies softmax + clipped-log loss on top.  fp32 like
        the template; on the GPU both ``tf.nn.xw_plus_b`` GEMMs (+ReLU) run on the f32 MFMA
        kernel with the bias / ReLU in its epilogue."""
        x = x.float()
        h = ops.dense(x, self.hid_w, self.hid_b, relu=True, layout="IO")
        return ops.dense(h, self.sm_w, self.sm_b, layout="IO")
