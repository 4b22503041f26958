"""MNIST IDX reader + DataSet semantics (main.py:43-44, worker.py:133,152-153)."""
import gzip
import os

import numpy as np
import pytest

from distributedtensorflowexample_amd.data import mnist


def test_idx_headers_of_reference_files():
    d = mnist.DEFAULT_DIR
    x = mnist.read_idx(os.path.join(d, mnist.TEST_IMAGES))
    y = mnist.read_idx(os.path.join(d, mnist.TEST_LABELS))
    t = mnist.read_idx(os.path.join(d, mnist.TRAIN_LABELS))
    assert x.shape == (10000, 28, 28) and x.dtype == np.uint8
    assert y.shape == (10000,) and t.shape == (60000,)
    assert set(np.unique(y)) == set(range(10))


def test_idx_bad_magic(tmp_path):
    p = tmp_path / "bad.gz"
    with gzip.open(p, "wb") as f:
        f.write(b"\x01\x02\x08\x01" + b"\x00" * 8)
    with pytest.raises(ValueError):
        mnist.read_idx(str(p))


def test_read_data_sets_splits_and_scaling():
    ds = mnist.read_data_sets(one_hot=True, seed=0)
    assert ds.synthetic_train  # train images are absent from the reference
    assert ds.train.num_examples == 55000 and ds.validation.num_examples == 5000
    assert ds.test.num_examples == 10000
    assert ds.test.images.shape == (10000, 784) and ds.test.images.dtype == np.float32
    assert 0.0 <= ds.test.images.min() and ds.test.images.max() <= 1.0
    assert ds.test.labels.shape == (10000, 10) and (ds.test.labels.sum(1) == 1).all()
    # the synthetic train images follow the REAL train labels
    raw = mnist.read_idx(os.path.join(mnist.DEFAULT_DIR, mnist.TRAIN_LABELS))
    assert (ds.validation.labels.argmax(1) == raw[:5000]).all()


def test_next_batch_epochs():
    x = np.arange(10, dtype=np.float32).reshape(10, 1)
    d = mnist.DataSet(x, np.arange(10) % 10, one_hot=False, seed=1, reshape=False)
    seen = []
    for _ in range(3):
        bx, by = d.next_batch(4)
        assert bx.shape == (4, 1)
        seen.extend(bx[:, 0].tolist())
    assert d.epochs_completed == 1
    assert sorted(seen[:10]) == list(range(10))  # first epoch covers every example once
