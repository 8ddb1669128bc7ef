"""HBM-resident array datasets (SURVEY.md R20/R21 "whole set resident in HBM").

MNIST is 47 MB as uint8 — trivially resident in 288 GB of HBM3E — so instead of a host pipeline
(decode -> batch -> copy per step, reference ``run_mnist_distributed.py:76-85``) the whole uint8
array is uploaded once and every batch is an on-device gather + normalisation (u8 -> compute dtype,
/255) with no host round trip and no per-step H2D copy.  ``repeat`` semantics (endless epochs),
optional per-epoch shuffle (device RNG) and per-replica sharding (``shard(n, i)``) match the
Dataset API.  On CPU the same class runs on host tensors (OneDeviceStrategy("/cpu:0")).
"""
from __future__ import annotations

import numpy as np
import torch


class DeviceArrayDataset:
    def __init__(self, images, labels, batch_size, device, dtype=None, shuffle=False, seed=0,
                 num_shards=1, shard_index=0, scale=1.0 / 255.0, drop_remainder=True):
        device = torch.device(device)
        imgs = torch.as_tensor(np.ascontiguousarray(images))
        labs = torch.as_tensor(np.ascontiguousarray(labels)).long()
        if num_shards > 1:                      # tf.data shard(): every num_shards-th element
            imgs, labs = imgs[shard_index::num_shards], labs[shard_index::num_shards]
        self.images = imgs.to(device)
        self.labels = labs.to(device)
        self.n = len(self.labels)
        self.batch_size = batch_size
        self.device = device
        self.dtype = dtype or (torch.bfloat16 if device.type == "cuda" else torch.float32)
        self.scale = scale
        self.shuffle = shuffle
        self.drop_remainder = drop_remainder
        self._gen = torch.Generator(device=device)
        self._gen.manual_seed(seed)
        self._order = None
        self._pos = 0
        self.epoch = 0
        if self.n < batch_size:
            raise ValueError(f"dataset of {self.n} examples < batch size {batch_size}")

    def _new_epoch(self):
        self._order = (torch.randperm(self.n, device=self.device, generator=self._gen)
                       if self.shuffle else torch.arange(self.n, device=self.device))
        self._pos = 0

    def __iter__(self):
        return self

    def __next__(self):
        if self._order is None:
            self._new_epoch()
        if self._pos + self.batch_size > self.n:
            if not self.drop_remainder and self._pos < self.n:
                idx = self._order[self._pos:]
                self._pos = self.n
                return self._gather(idx)
            self.epoch += 1
            self._new_epoch()
        idx = self._order[self._pos:self._pos + self.batch_size]
        self._pos += self.batch_size
        return self._gather(idx)

    def _gather(self, idx):
        if (self.device.type == "cuda" and self.images.dtype == torch.uint8
                and self.dtype in (torch.bfloat16, torch.float32)
                and (self.images[0].numel() % 8) == 0):
            # u8 decode + /255 fused into the gather, one HIP kernel per batch
            from ..ops import native
            B = idx.numel()
            x = torch.empty(B, *self.images.shape[1:], device=self.device, dtype=self.dtype)
            native.kernels().gather_u8_scale(
                self.images.data_ptr(), idx.contiguous().data_ptr(), x.data_ptr(), B,
                self.images[0].numel(), float(self.scale), int(self.dtype == torch.bfloat16),
                torch.cuda.current_stream().cuda_stream)
            return x, self.labels.index_select(0, idx)
        x = self.images.index_select(0, idx).to(self.dtype)
        if self.scale != 1.0:
            x = x * self.scale
        return x, self.labels.index_select(0, idx)
