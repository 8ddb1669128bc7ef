"""Stock PyTorch-ROCm ResNet-50 — the comparator for the north-star benchmark.

BASELINE.md: the reference publishes no GPU/ResNet number, so the comparator is idiomatic
stock PyTorch on the same MI355X: ``nn.Conv2d``/``nn.BatchNorm2d`` (MIOpen), channels_last,
bf16 autocast, ``torch.optim.SGD(momentum, foreach)``, DDP for N>1.  Same architecture
(v1.5), same batch, same synthetic data as :mod:`bench`.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class _Block(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                      nn.BatchNorm2d(cout))

    def forward(self, x):
        sc = x if self.down is None else self.down(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + sc)


class TorchResNet50(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64),
                                  nn.ReLU(inplace=True), nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], 64
        for si, (n, w) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
            for bi in range(n):
                blocks.append(_Block(cin, w, 2 if (bi == 0 and si > 0) else 1))
                cin = w * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        y = self.blocks(self.stem(x))
        y = torch.flatten(nn.functional.adaptive_avg_pool2d(y, 1), 1)
        return self.fc(y)
