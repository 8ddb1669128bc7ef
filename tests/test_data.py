"""Input pipeline: tf.data-style Dataset semantics (reference ``dataset.py`` /
``run_mnist_distributed.py:77-85``: ``repeat().batch(128).prefetch``), the native C++ batch
prefetcher, MNIST idx header checks (``dataset.py:30-59``) and the offline synthetic fallback."""
import itertools
import os

import numpy as np
import pytest

from distributedtensorflow_amd.data import Dataset, mnist
from distributedtensorflow_amd.data.dataset import Iterator


def test_from_tensor_slices_batch_repeat():
    a = np.arange(10)
    b = np.arange(10) * 2
    ds = Dataset.from_tensor_slices((a, b)).batch(4)
    batches = list(ds)
    assert [len(x) for x, _ in batches] == [4, 4, 2]
    np.testing.assert_array_equal(batches[2][1], [16, 18])
    assert [len(x) for x, _ in Dataset.from_tensor_slices((a, b)).batch(4, True)] == [4, 4]
    rep = list(itertools.islice(iter(Dataset.from_tensor_slices(a).repeat()), 25))
    assert rep == list(range(10)) * 2 + list(range(5))
    assert list(Dataset.range(3).repeat(2)) == [0, 1, 2, 0, 1, 2]


def test_map_filter_take_skip_shard_zip():
    ds = Dataset.range(20).map(lambda x: x * 3).filter(lambda x: x % 2 == 0)
    assert list(ds.take(3)) == [0, 6, 12]
    assert list(ds.skip(8)) == [48, 54]
    assert list(Dataset.range(10).shard(3, 1)) == [1, 4, 7]
    z = Dataset.zip((Dataset.range(3), Dataset.range(3).map(lambda x: -x)))
    assert list(z) == [(0, 0), (1, -1), (2, -2)]
    assert Dataset.range(7).cardinality() == 7
    g = Dataset.from_generator(lambda: iter([1, 2, 3]))
    assert list(g) == [1, 2, 3] and list(g) == [1, 2, 3]      # re-iterable


def test_shuffle_is_permutation_and_seeded():
    a = list(Dataset.range(100).shuffle(30, seed=1))
    b = list(Dataset.range(100).shuffle(30, seed=1))
    assert sorted(a) == list(range(100)) and a == b and a != list(range(100))


def test_prefetch_thread_preserves_order_and_errors():
    assert list(Dataset.range(50).prefetch(4)) == list(range(50))

    def bad():
        yield 1
        raise ValueError("boom")
    with pytest.raises(ValueError, match="boom"):
        list(Dataset.from_generator(bad).prefetch(2))


def test_initializable_iterator():
    it = Iterator.from_structure()
    init_a = it.make_initializer(Dataset.range(3))
    init_b = it.make_initializer(Dataset.range(10, 12))
    init_a()
    assert [next(it) for _ in range(3)] == [0, 1, 2]
    init_b()
    assert it.get_next() == 10


def test_native_prefetcher_covers_epoch_and_shards():
    n, dim = 64, 12
    imgs = (np.arange(n * dim) % 256).astype(np.uint8).reshape(n, dim)
    labels = np.arange(n)
    ds = Dataset.range(1).with_native_prefetch(imgs, labels, 16, shuffle=True, seed=3, threads=3)
    it = iter(ds)
    seen = []
    for _ in range(n // 16):
        x, y = next(it)
        assert x.shape == (16, dim) and x.dtype == np.float32
        np.testing.assert_allclose(x, imgs[y].astype(np.float32) / 255.0)
        seen += list(y)
    assert sorted(seen) == list(range(n))                       # one epoch = a permutation
    it.close()
    parts = []
    for k in range(2):
        it = iter(Dataset.range(1).with_native_prefetch(imgs, labels, 8, shard_index=k,
                                                        num_shards=2))
        parts.append(set(int(v) for _ in range(n // 16) for v in next(it)[1]))
        it.close()
    assert parts[0].isdisjoint(parts[1]) and len(parts[0] | parts[1]) == n


def test_mnist_headers_and_synthetic(tmp_path):
    imgs, labels = mnist.load_arrays(str(tmp_path), "test")
    assert imgs.shape == (10000, 784) and imgs.dtype == np.uint8
    assert labels.shape == (10000,) and set(np.unique(labels)) == set(range(10))
    mnist.check_image_file_header(os.path.join(tmp_path, "t10k-images-idx3-ubyte"))
    with pytest.raises(ValueError, match="Invalid magic number 2049"):
        mnist.check_image_file_header(os.path.join(tmp_path, "t10k-labels-idx1-ubyte"))
    bad = tmp_path / "bad"
    from distributedtensorflow_amd.io.native import lib
    lib().write_idx(str(bad), np.zeros((2, 27, 28), np.uint8))
    with pytest.raises(ValueError, match="Expected 28x28"):
        mnist.check_image_file_header(str(bad))
    ds = mnist.test(str(tmp_path))
    x, y = next(iter(ds.batch(5)))
    assert x.shape == (5, 784) and x.dtype == np.float32 and x.max() <= 1.0
    assert mnist.synthetic_mnist(4, seed=0)[0].tobytes() == mnist.synthetic_mnist(4, seed=0)[0].tobytes()


def test_read_data_sets_next_batch(tmp_path):
    d = mnist.read_data_sets(str(tmp_path), one_hot=True, validation_size=100)
    assert d.validation.num_examples == 100 and d.train.num_examples == 59900
    x, y = d.train.next_batch(32)
    assert x.shape == (32, 784) and y.shape == (32, 10) and np.all(y.sum(1) == 1)
