"""MNIST input pipeline (``tensorflow.examples.tutorials.mnist.input_data``).

The reference loads MNIST in every process with
``input_data.read_data_sets('MNIST_data', one_hot=True)`` (main.py:43-44) and
feeds ``mnist.train.next_batch(100)`` per step (worker.py:133) and the whole
test set for evaluation (worker.py:152-153).  Same API here:

* :func:`read_idx` -- IDX (ubyte) reader, gzip or raw, big-endian header.
* :class:`DataSet` -- images scaled to [0, 1] float32 [N, 784], labels one-hot
  float32 [N, 10] or int; ``next_batch`` reshuffles at every epoch boundary
  and stitches the epoch's tail with the next epoch's head, like TF's.
* :func:`read_data_sets` -- train 55,000 / validation 5,000 / test 10,000.

Offline caveat: the reference ships the test set and the train LABELS but not
the train images (.MISSING_LARGE_BLOBS:1).  When they are absent the train
images are synthesized for the real train labels: each image is the
real-test-set mean image of its class, randomly shifted by up to 2 pixels,
plus clipped Gaussian noise.  ``DataSets.synthetic_train`` says so.  Test
accuracy is always measured on the real test set.
"""
from __future__ import annotations

import gzip
import os
import struct
from collections import namedtuple

import numpy as np

DEFAULT_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "assets", "MNIST_data")
TRAIN_IMAGES = "train-images-idx3-ubyte.gz"
TRAIN_LABELS = "train-labels-idx1-ubyte.gz"
TEST_IMAGES = "t10k-images-idx3-ubyte.gz"
TEST_LABELS = "t10k-labels-idx1-ubyte.gz"

_IDX_TYPES = {0x08: np.uint8, 0x09: np.int8, 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4", 0x0E: ">f8"}


def read_idx(path):
    """Read an IDX file (optionally gzipped) into a numpy array."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    if len(data) < 4 or data[0] != 0 or data[1] != 0:
        raise ValueError("%s: not an IDX file (bad magic)" % path)
    dtype = _IDX_TYPES.get(data[2])
    if dtype is None:
        raise ValueError("%s: unknown IDX element type 0x%02x" % (path, data[2]))
    ndim = data[3]
    dims = struct.unpack(">" + "I" * ndim, data[4:4 + 4 * ndim])
    arr = np.frombuffer(data, dtype=dtype, offset=4 + 4 * ndim)
    n = int(np.prod(dims))
    if arr.size < n:
        raise ValueError("%s: truncated (%d of %d elements)" % (path, arr.size, n))
    return arr[:n].reshape(dims)


def dense_to_one_hot(labels, num_classes=10):
    out = np.zeros((labels.shape[0], num_classes), dtype=np.float32)
    out[np.arange(labels.shape[0]), labels.astype(np.int64)] = 1.0
    return out


class DataSet:
    def __init__(self, images, labels, one_hot=True, seed=None, dtype=np.float32, reshape=True):
        images = np.asarray(images)
        if reshape and images.ndim == 3:
            images = images.reshape(images.shape[0], -1)
        if images.dtype == np.uint8 and dtype == np.float32:
            images = images.astype(np.float32) * (1.0 / 255.0)
        self._images = images.astype(dtype, copy=False)
        labels = np.asarray(labels)
        if one_hot and labels.ndim == 1:
            labels = dense_to_one_hot(labels)
        self._labels = labels
        if self._images.shape[0] != self._labels.shape[0]:
            raise ValueError("images/labels count mismatch")
        self._num_examples = self._images.shape[0]
        self._epochs_completed = 0
        self._index_in_epoch = 0
        self._rng = np.random.RandomState(seed)  # None: unseeded, like the reference

    images = property(lambda self: self._images)
    labels = property(lambda self: self._labels)
    num_examples = property(lambda self: self._num_examples)
    epochs_completed = property(lambda self: self._epochs_completed)

    def _shuffle(self):
        perm = self._rng.permutation(self._num_examples)
        self._images = self._images[perm]
        self._labels = self._labels[perm]

    def next_batch(self, batch_size, shuffle=True):
        start = self._index_in_epoch
        if self._epochs_completed == 0 and start == 0 and shuffle:
            self._shuffle()
        if start + batch_size > self._num_examples:
            self._epochs_completed += 1
            rest = self._num_examples - start
            imgs_rest, labs_rest = self._images[start:], self._labels[start:]
            if shuffle:
                self._shuffle()
            start, self._index_in_epoch = 0, batch_size - rest
            end = self._index_in_epoch
            return (np.concatenate((imgs_rest, self._images[start:end]), 0),
                    np.concatenate((labs_rest, self._labels[start:end]), 0))
        self._index_in_epoch += batch_size
        end = self._index_in_epoch
        return self._images[start:end], self._labels[start:end]


DataSets = namedtuple("DataSets", ["train", "validation", "test", "synthetic_train"])


def synthesize_images(labels, test_images, test_labels, seed=0, noise=0.25, max_shift=2):
    """Train images for real labels: class-mean test image, shifted, + noise (uint8)."""
    rng = np.random.RandomState(seed)
    timg = test_images.reshape(-1, 28, 28).astype(np.float32)
    protos = np.stack([timg[test_labels == c].mean(0) for c in range(10)])
    n = labels.shape[0]
    out = np.empty((n, 28, 28), dtype=np.uint8)
    chunk = 8192
    for s in range(0, n, chunk):
        lab = labels[s:s + chunk]
        img = protos[lab]
        dx, dy = rng.randint(-max_shift, max_shift + 1, size=(2, lab.shape[0]))
        for k in range(lab.shape[0]):
            img[k] = np.roll(np.roll(img[k], dx[k], 0), dy[k], 1)
        img = img + rng.normal(0.0, noise * 255.0, size=img.shape)
        out[s:s + chunk] = np.clip(img, 0, 255).astype(np.uint8)
    return out


def read_data_sets(train_dir=None, one_hot=True, validation_size=5000, seed=None,
                   synthetic_seed=0):
    d = train_dir or DEFAULT_DIR
    test_images = read_idx(os.path.join(d, TEST_IMAGES))
    test_labels = read_idx(os.path.join(d, TEST_LABELS))
    train_labels = read_idx(os.path.join(d, TRAIN_LABELS))
    tip = os.path.join(d, TRAIN_IMAGES)
    synthetic = not os.path.exists(tip)
    if synthetic:
        train_images = synthesize_images(train_labels, test_images, test_labels, synthetic_seed)
    else:  # pragma: no cover - file not shipped with the reference
        train_images = read_idx(tip)
    if not 0 <= validation_size <= len(train_images):
        raise ValueError("validation_size must be in [0, %d]" % len(train_images))
    val = DataSet(train_images[:validation_size], train_labels[:validation_size], one_hot, seed)
    train = DataSet(train_images[validation_size:], train_labels[validation_size:], one_hot, seed)
    test = DataSet(test_images, test_labels, one_hot, seed)
    return DataSets(train, val, test, synthetic)
