"""Device-resident synthetic datasets for benchmarks (no network: BASELINE 'synthetic' data).

``SyntheticImageNet`` yields NHWC bf16 ``[B,224,224,3]`` images + int64 labels already in HBM
(a fixed pool of batches generated once on the device, cycled), so the timed loop measures the
training step, not host I/O — the same protocol as tf_cnn_benchmarks' ``--use_synthetic_data``.
``SyntheticMLM`` yields BERT masked-LM batches (token ids, segment ids, attention mask, masked
positions / labels).
"""
from __future__ import annotations

import torch


class SyntheticImageNet:
    def __init__(self, batch_size, image_size=224, num_classes=1000, device="cuda",
                 dtype=torch.bfloat16, pool=2, seed=1234, channels_last=True):
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        shape = (batch_size, image_size, image_size, 3) if channels_last else \
            (batch_size, 3, image_size, image_size)
        self.images = [torch.randn(shape, device=device, generator=g).to(dtype)
                       for _ in range(pool)]
        self.labels = [torch.randint(0, num_classes, (batch_size,), device=device, generator=g)
                       for _ in range(pool)]
        self.i = 0

    def __iter__(self):
        return self

    def __next__(self):
        k = self.i % len(self.images)
        self.i += 1
        return self.images[k], self.labels[k]


class SyntheticMLM:
    def __init__(self, batch_size, seq_len=128, vocab_size=30522, max_predictions=20,
                 device="cuda", seed=1234, pool=2):
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        self.batches = []
        for _ in range(pool):
            ids = torch.randint(0, vocab_size, (batch_size, seq_len), device=device, generator=g)
            seg = torch.zeros_like(ids)
            seg[:, seq_len // 2:] = 1
            mask = torch.ones_like(ids)
            pos = torch.stack([torch.randperm(seq_len, device=device, generator=g)[:max_predictions]
                               for _ in range(batch_size)])
            lab = torch.randint(0, vocab_size, (batch_size, max_predictions), device=device,
                                generator=g)
            self.batches.append({"input_ids": ids, "segment_ids": seg, "input_mask": mask,
                                 "masked_lm_positions": pos, "masked_lm_ids": lab})
        self.i = 0

    def __iter__(self):
        return self

    def __next__(self):
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b
