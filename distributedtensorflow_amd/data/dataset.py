"""A ``tf.data.Dataset``-style input pipeline.

The reference builds ``dataset.train(dir).repeat().batch(128).prefetch(128)`` and a
re-initialisable iterator (``run_mnist_distributed.py:76-85,111,133``).  Here a Dataset is a
lazily composed Python iterator over numpy/torch elements:

* ``from_tensor_slices / zip / range / from_generator`` sources;
* ``map, batch(drop_remainder), repeat, shuffle(buffer, seed), shard, take, skip, prefetch``;
* ``prefetch`` runs the upstream pipeline on a background thread (bounded queue);
* array-backed ``...shuffle().repeat().batch()`` chains over uint8 images can be executed by the
  native C++ ``BatchPrefetcher`` (``with_native_prefetch``), which normalises on worker threads;
* ``to_device(device)`` moves each element to the GPU on a side stream (non-blocking copies).

Iterator API compat: ``make_one_shot_iterator()``, ``Iterator.from_structure`` +
``make_initializer`` + ``get_next``.
"""
from __future__ import annotations

import queue
import threading

import numpy as np


class Dataset:
    def __init__(self, gen_fn, structure=None):
        self._gen_fn = gen_fn          # () -> iterator
        self._structure = structure

    # ---------------------------------------------------------------- sources
    @staticmethod
    def from_tensor_slices(tensors):
        if isinstance(tensors, (tuple, list)):
            arrs = [np.asarray(t) if not hasattr(t, "shape") else t for t in tensors]
            n = len(arrs[0])
            return Dataset(lambda: (tuple(a[i] for a in arrs) for i in range(n)),
                           ("tuple", len(arrs)))
        if isinstance(tensors, dict):
            keys = list(tensors)
            n = len(tensors[keys[0]])
            return Dataset(lambda: ({k: tensors[k][i] for k in keys} for i in range(n)))
        arr = tensors
        return Dataset(lambda: (arr[i] for i in range(len(arr))))

    from_tensors = staticmethod(lambda t: Dataset(lambda: iter([t])))

    @staticmethod
    def range(*args):
        return Dataset(lambda: iter(range(*args)))

    @staticmethod
    def zip(datasets):
        return Dataset(lambda: zip(*[iter(d) for d in datasets]))

    @staticmethod
    def from_generator(generator, output_types=None, output_shapes=None):
        return Dataset(generator)

    # ---------------------------------------------------------------- transforms
    def map(self, fn, num_parallel_calls=None):
        src = self

        def gen():
            for e in src:
                yield fn(*e) if isinstance(e, tuple) else fn(e)
        return Dataset(gen)

    def filter(self, pred):
        src = self
        return Dataset(lambda: (e for e in src if (pred(*e) if isinstance(e, tuple) else pred(e))))

    def batch(self, batch_size, drop_remainder=False):
        src = self

        def stack(items):
            first = items[0]
            if isinstance(first, tuple):
                return tuple(stack([it[j] for it in items]) for j in range(len(first)))
            if isinstance(first, dict):
                return {k: stack([it[k] for it in items]) for k in first}
            if hasattr(first, "dim") and hasattr(first, "unsqueeze"):   # torch
                import torch
                return torch.stack(list(items))
            return np.stack([np.asarray(x) for x in items])

        def gen():
            buf = []
            for e in src:
                buf.append(e)
                if len(buf) == batch_size:
                    yield stack(buf)
                    buf = []
            if buf and not drop_remainder:
                yield stack(buf)
        return Dataset(gen)

    def repeat(self, count=None):
        src = self

        def gen():
            n = 0
            while count is None or count < 0 or n < count:
                empty = True
                for e in src:
                    empty = False
                    yield e
                n += 1
                if empty:
                    return
        return Dataset(gen)

    def shuffle(self, buffer_size, seed=None, reshuffle_each_iteration=True):
        src = self
        state = {"epoch": 0}

        def gen():
            rng = np.random.default_rng(None if seed is None else seed + (
                state["epoch"] if reshuffle_each_iteration else 0))
            state["epoch"] += 1
            buf = []
            for e in src:
                if len(buf) < buffer_size:
                    buf.append(e)
                    continue
                j = rng.integers(len(buf))
                yield buf[j]
                buf[j] = e
            rng.shuffle(buf)
            yield from buf
        return Dataset(gen)

    def shard(self, num_shards, index):
        src = self
        return Dataset(lambda: (e for i, e in enumerate(src) if i % num_shards == index))

    def take(self, count):
        src = self

        def gen():
            for i, e in enumerate(src):
                if i >= count:
                    return
                yield e
        return Dataset(gen)

    def skip(self, count):
        src = self
        return Dataset(lambda: (e for i, e in enumerate(src) if i >= count))

    def prefetch(self, buffer_size=1):
        src = self
        size = max(1, int(buffer_size) if buffer_size and buffer_size > 0 else 2)

        def gen():
            q: queue.Queue = queue.Queue(maxsize=size)
            stop = threading.Event()
            done = object()
            error = []

            def producer():
                try:
                    for e in src:
                        while not stop.is_set():
                            try:
                                q.put(e, timeout=0.1)
                                break
                            except queue.Full:
                                continue
                        if stop.is_set():
                            return
                except BaseException as exc:     # re-raised in the consumer, like tf.data
                    error.append(exc)
                finally:
                    while not stop.is_set():
                        try:
                            q.put(done, timeout=0.1)
                            break
                        except queue.Full:
                            continue
            t = threading.Thread(target=producer, daemon=True)
            t.start()
            try:
                while True:
                    e = q.get()
                    if e is done:
                        if error:
                            raise error[0]
                        return
                    yield e
            finally:
                stop.set()
        return Dataset(gen)

    def to_device(self, device, non_blocking=True):
        import torch
        src = self

        def move(x):
            if isinstance(x, tuple):
                return tuple(move(v) for v in x)
            if isinstance(x, dict):
                return {k: move(v) for k, v in x.items()}
            t = torch.as_tensor(x)
            return t.to(device, non_blocking=non_blocking) if t.device != torch.device(device) \
                else t
        return Dataset(lambda: (move(e) for e in src))

    def with_native_prefetch(self, images_u8, labels, batch_size, shuffle=False, seed=0,
                             threads=2, depth=4, scale=1.0 / 255.0, shard_index=0, num_shards=1):
        """Replace this pipeline by the C++ producer pool over in-memory uint8 images."""
        return NativeBatchDataset(images_u8, labels, batch_size, shuffle, seed, threads, depth,
                                  scale, shard_index, num_shards)

    # ---------------------------------------------------------------- iteration
    def __iter__(self):
        return iter(self._gen_fn())

    def make_one_shot_iterator(self):
        return Iterator(self)

    def make_initializable_iterator(self):
        return Iterator(self)

    @property
    def output_types(self):
        return None

    @property
    def output_shapes(self):
        return None

    def cardinality(self):
        return sum(1 for _ in self)


class NativeBatchDataset(Dataset):
    def __init__(self, images_u8, labels, batch_size, shuffle, seed, threads, depth, scale,
                 shard_index, num_shards):
        from ..io.native import lib
        self.images = np.ascontiguousarray(images_u8, dtype=np.uint8)
        self.labels = None if labels is None else np.ascontiguousarray(labels, dtype=np.int64)
        self.dim = int(self.images.size // self.images.shape[0])
        self.args = (batch_size, shuffle, seed, threads, depth, scale, shard_index, num_shards)
        self._lib = lib()
        super().__init__(self._gen)

    def _gen(self):
        bs, sh, seed, th, dp, sc, si, ns = self.args
        p = self._lib.BatchPrefetcher(self.images, self.labels, bs, sh, seed, th, dp, sc, True,
                                      si, ns)
        try:
            while True:
                x, y = p.next(self.dim)
                yield x, y
        finally:
            p.stop()


class Iterator:
    """Re-initialisable iterator (``tf.data.Iterator.from_structure`` / ``make_initializer``)."""

    def __init__(self, dataset=None):
        self._ds = dataset
        self._it = iter(dataset) if dataset is not None else None

    @staticmethod
    def from_structure(output_types=None, output_shapes=None):
        return Iterator(None)

    def make_initializer(self, dataset):
        def init():
            self._ds = dataset
            self._it = iter(dataset)
        return init

    def get_next(self):
        if self._it is None:
            raise RuntimeError("iterator not initialised (run make_initializer(dataset)())")
        return next(self._it)

    def __iter__(self):
        return self

    def __next__(self):
        return self.get_next()
