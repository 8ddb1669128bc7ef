"""TF checkpoint V2 tensor bundles (``.index`` SSTable + ``.data-K-of-N``) via the native C++
writer/reader (csrc/native/bundle.cpp).  numpy in, numpy out."""
from __future__ import annotations

import numpy as np

from .native import lib

# TF DataType enum <-> numpy
_NP2TF = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3,
          np.dtype(np.uint8): 4, np.dtype(np.int16): 5, np.dtype(np.int8): 6,
          np.dtype(np.int64): 9, np.dtype(np.bool_): 10, np.dtype(np.float16): 19}
_TF2NP = {v: k for k, v in _NP2TF.items()}
DT_BFLOAT16 = 14


def write_bundle(prefix: str, tensors: dict, num_shards: int = 1, shard_of=None):
    """tensors: {name: np.ndarray (or torch tensor)}; ``shard_of(name) -> k`` for sharded saves."""
    w = lib().BundleWriter(prefix, num_shards)
    for name in sorted(tensors):
        arr = tensors[name]
        if hasattr(arr, "detach"):
            import torch
            t = arr.detach().cpu()
            if t.dtype == torch.bfloat16:
                raw = np.ascontiguousarray(t.view(torch.int16).numpy())
                w.add(name, DT_BFLOAT16, list(t.shape), raw, shard_of(name) if shard_of else 0)
                continue
            arr = t.numpy()
        arr = np.asarray(arr, order="C")          # (ascontiguousarray would promote 0-d to [1])
        if arr.dtype not in _NP2TF:
            raise TypeError(f"unsupported dtype {arr.dtype} for {name}")
        w.add(name, _NP2TF[arr.dtype], list(arr.shape), arr.reshape(-1) if arr.ndim else
              arr.reshape(1), shard_of(name) if shard_of else 0)
    w.finish()


class BundleReader:
    def __init__(self, prefix: str):
        self._r = lib().BundleReader(prefix)

    def keys(self):
        return list(self._r.keys())

    def entry(self, name):
        return self._r.entry(name)

    def get_variable_to_shape_map(self):
        return {k: list(self._r.entry(k)["shape"]) for k in self.keys()}

    def get_tensor(self, name) -> np.ndarray:
        e = self._r.entry(name)
        raw = self._r.read(name)
        if e["dtype"] == DT_BFLOAT16:
            u16 = np.frombuffer(raw, dtype=np.uint16).astype(np.uint32) << 16
            return u16.view(np.float32).reshape(e["shape"])
        dt = _TF2NP[e["dtype"]]
        return np.frombuffer(raw, dtype=dt).reshape(e["shape"]).copy()

    def has_tensor(self, name):
        return name in set(self.keys())
