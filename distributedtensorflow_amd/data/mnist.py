"""MNIST in idx format (reference ``dataset.py``).

* header validation as the reference: images magic 2051 and 28x28, labels magic 2049
  (big-endian uint32 words, ``dataset.py:30-59``); parsing in C++ (``_dtf_native.read_idx``);
* ``train(dir)`` / ``test(dir)`` -> Dataset of ``(float32[784] in [0,1], int32 label)``;
* ``download(dir, filename)``: uses existing files (plain or ``.gz``) in ``dir``; otherwise tries
  the CVDF mirror, and when there is no network (this environment, the GPU boxes) writes a
  DETERMINISTIC SYNTHETIC stand-in with the same idx format/shape (10 learnable class
  prototypes + noise) and says so — numbers on it are "synthetic MNIST-shaped data".
* ``read_data_sets(dir, one_hot)`` — the tutorials ``input_data`` API used by
  ``templates/00_mnist_replica.py:92,249`` (train/validation/test with ``next_batch``).
"""
from __future__ import annotations

import gzip
import os
import shutil
import tempfile
import warnings

import numpy as np

from ..io.native import lib
from .dataset import Dataset

MIRROR = "https://storage.googleapis.com/cvdf-datasets/mnist/"
FILES = {"train": ("train-images-idx3-ubyte", "train-labels-idx1-ubyte", 60000),
         "test": ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte", 10000)}


def _read32_be(b, off):
    return int.from_bytes(b[off:off + 4], "big")


def check_image_file_header(filename):
    with open(filename, "rb") as f:
        h = f.read(16)
    magic, rows, cols = _read32_be(h, 0), _read32_be(h, 8), _read32_be(h, 12)
    if magic != 2051:
        raise ValueError(f"Invalid magic number {magic} in MNIST file {filename}")
    if rows != 28 or cols != 28:
        raise ValueError(f"Invalid MNIST file {filename}: Expected 28x28 images, found "
                         f"{rows}x{cols}")


def check_labels_file_header(filename):
    with open(filename, "rb") as f:
        h = f.read(8)
    magic = _read32_be(h, 0)
    if magic != 2049:
        raise ValueError(f"Invalid magic number {magic} in MNIST file {filename}")


def synthetic_mnist(n, seed):
    """Deterministic MNIST-shaped data: class prototypes (smooth blobs) + noise, uint8."""
    rng = np.random.default_rng(1234)            # prototypes shared by train and test
    yy, xx = np.mgrid[0:28, 0:28]
    protos = []
    for c in range(10):
        img = np.zeros((28, 28))
        for _ in range(3):
            cy, cx = rng.uniform(6, 22, 2)
            s = rng.uniform(2.0, 4.5)
            img += np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
        protos.append(img / img.max())
    protos = np.stack(protos).astype(np.float32)
    # all 25 (dy, dx) shifts of every prototype, then gather (vectorised)
    shifted = np.stack([np.roll(protos, (dy, dx), axis=(1, 2))
                        for dy in range(-2, 3) for dx in range(-2, 3)], axis=1)  # [10,25,28,28]
    r = np.random.default_rng(seed)
    labels = r.integers(0, 10, n).astype(np.uint8)
    which = r.integers(0, 25, n)
    imgs = shifted[labels, which] * r.uniform(0.7, 1.0, (n, 1, 1)).astype(np.float32)
    imgs += r.normal(0, 0.08, imgs.shape).astype(np.float32)
    return (np.clip(imgs, 0, 1) * 255).astype(np.uint8), labels


def _write_synthetic(directory, split):
    """Write atomically (tmp + rename) so concurrent worker processes never read partial files."""
    img_name, lab_name, n = FILES[split]
    imgs, labels = synthetic_mnist(n, seed=0 if split == "train" else 1)
    for name, arr in ((img_name, imgs), (lab_name, labels)):
        final = os.path.join(directory, name)
        tmp = f"{final}.tmp.{os.getpid()}"
        lib().write_idx(tmp, arr)
        os.replace(tmp, final)


def download(directory, filename, allow_synthetic=True):
    """Return the path of ``filename`` in ``directory``, fetching / synthesising if absent."""
    path = os.path.join(directory, filename)
    if os.path.exists(path):
        return path
    os.makedirs(directory, exist_ok=True)
    gz = path + ".gz"
    if os.path.exists(gz):
        with gzip.open(gz, "rb") as fi, open(path, "wb") as fo:
            shutil.copyfileobj(fi, fo)
        return path
    try:
        if os.environ.get("DTF_OFFLINE", "1") == "1":
            raise ConnectionError("offline (set DTF_OFFLINE=0 to try the CVDF mirror)")
        import urllib.request
        fd, tmp = tempfile.mkstemp(suffix=".gz")
        os.close(fd)
        with urllib.request.urlopen(MIRROR + filename + ".gz", timeout=10) as r, \
                open(tmp, "wb") as fo:
            shutil.copyfileobj(r, fo)
        with gzip.open(tmp, "rb") as fi, open(path, "wb") as fo:
            shutil.copyfileobj(fi, fo)
        os.remove(tmp)
        return path
    except Exception as e:  # no network here
        if not allow_synthetic:
            raise
        split = "train" if filename.startswith("train") else "test"
        warnings.warn(f"MNIST download failed ({type(e).__name__}); writing deterministic "
                      f"synthetic MNIST-shaped {split} data to {directory}")
        _write_synthetic(directory, split)
        return path


def load_arrays(directory, split="train"):
    img_name, lab_name, _ = FILES[split]
    ip = download(directory, img_name)
    lp = download(directory, lab_name)
    check_image_file_header(ip)
    check_labels_file_header(lp)
    _, imgs = lib().read_idx(ip)
    _, labels = lib().read_idx(lp)
    if len(imgs) != len(labels):
        raise ValueError("image / label count mismatch")
    return imgs.reshape(len(imgs), 784), labels.astype(np.int32)


def dataset(directory, split):
    imgs, labels = load_arrays(directory, split)
    images = Dataset.from_tensor_slices(imgs).map(lambda x: x.astype(np.float32) / 255.0)
    lab = Dataset.from_tensor_slices(labels).map(lambda y: np.int32(y))
    ds = Dataset.zip((images, lab))
    ds.arrays = (imgs, labels)
    return ds


def train(directory):
    return dataset(directory, "train")


def test(directory):
    return dataset(directory, "test")


# ----------------------------------------------------------------------------- input_data API

class DataSet:
    def __init__(self, images_u8, labels, one_hot=False, seed=0):
        self.images = images_u8.reshape(len(images_u8), 784).astype(np.float32) / 255.0
        self.labels = (np.eye(10, dtype=np.float32)[labels] if one_hot else labels.astype(np.int64))
        self.num_examples = len(self.images)
        self._rng = np.random.default_rng(seed)
        self._perm = self._rng.permutation(self.num_examples)
        self._pos = 0
        self.epochs_completed = 0

    def next_batch(self, batch_size):
        if self._pos + batch_size > self.num_examples:
            self.epochs_completed += 1
            self._perm = self._rng.permutation(self.num_examples)
            self._pos = 0
        idx = self._perm[self._pos:self._pos + batch_size]
        self._pos += batch_size
        return self.images[idx], self.labels[idx]


class Datasets:
    def __init__(self, train, validation, test):
        self.train, self.validation, self.test = train, validation, test


def read_data_sets(train_dir, one_hot=False, validation_size=5000, seed=0):
    tr_i, tr_l = load_arrays(train_dir, "train")
    te_i, te_l = load_arrays(train_dir, "test")
    return Datasets(DataSet(tr_i[validation_size:], tr_l[validation_size:], one_hot, seed),
                    DataSet(tr_i[:validation_size], tr_l[:validation_size], one_hot, seed + 1),
                    DataSet(te_i, te_l, one_hot, seed + 2))
