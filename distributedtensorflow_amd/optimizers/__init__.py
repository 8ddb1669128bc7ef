"""TF1-compatible optimizers on flat fp32 buffers with fused HIP updates."""
from .base import FlatSpace, Optimizer, default_decay_filter, tf_adam_lr_t
from .optimizers import (SGD, AdagradOptimizer, AdamOptimizer, GradientDescentOptimizer,
                         LAMBOptimizer, MomentumOptimizer, clip_by_global_norm_, cosine_decay,
                         piecewise_constant, polynomial_decay)
from .sync_replicas import SyncReplicasOptimizer

__all__ = ["FlatSpace", "Optimizer", "default_decay_filter", "tf_adam_lr_t", "SGD",
           "AdagradOptimizer", "AdamOptimizer", "GradientDescentOptimizer", "LAMBOptimizer",
           "MomentumOptimizer", "SyncReplicasOptimizer", "clip_by_global_norm_", "cosine_decay",
           "piecewise_constant", "polynomial_decay"]
