"""Dataset loaders and augmentation (reference ``python/hetu/data.py:5-338``).

No network access is assumed: loaders read the standard on-disk formats
(MNIST ``mnist.pkl.gz`` / idx files, CIFAR-10/100 python pickles) from a
directory when present, and otherwise fall back to deterministic synthetic
arrays of the same shapes (``synthetic=True`` or files missing).
"""
from __future__ import annotations

import gzip
import os
import pickle

import numpy as np


def _onehot(y, n):
    out = np.zeros((len(y), n), dtype=np.float32)
    out[np.arange(len(y)), np.asarray(y, dtype=np.int64)] = 1.0
    return out


def synthetic_classification(n, shape, num_classes, seed=0, onehot=True):
    rng = np.random.RandomState(seed)
    x = rng.standard_normal((n,) + tuple(shape)).astype(np.float32)
    y = rng.randint(0, num_classes, size=n)
    return x, (_onehot(y, num_classes) if onehot else y.astype(np.float32))


def mnist(path='datasets/mnist.pkl.gz', onehot=True, synthetic=None):
    """Returns ((train_x, train_y), (valid_x, valid_y), (test_x, test_y)), x [N, 784]."""
    if synthetic or not os.path.exists(path):
        tr = synthetic_classification(6000, (784,), 10, 0, onehot)
        va = synthetic_classification(1000, (784,), 10, 1, onehot)
        te = synthetic_classification(1000, (784,), 10, 2, onehot)
        return tr, va, te
    with gzip.open(path, 'rb') as f:
        sets = pickle.load(f, encoding='latin1')
    out = []
    for x, y in sets:
        out.append((x.astype(np.float32), _onehot(y, 10) if onehot else y.astype(np.float32)))
    return tuple(out)


def normalize_cifar(num_class=10, onehot=True, path=None, synthetic=None):
    """CIFAR-10/100 as float32 NCHW normalised by per-channel mean/std."""
    path = path or 'datasets/cifar-%d-python' % num_class
    if synthetic or not os.path.exists(path):
        xtr, ytr = synthetic_classification(5000, (3, 32, 32), num_class, 3, onehot)
        xte, yte = synthetic_classification(1000, (3, 32, 32), num_class, 4, onehot)
        return xtr, ytr, xte, yte
    def _load(fname):
        with open(os.path.join(path, fname), 'rb') as f:
            d = pickle.load(f, encoding='latin1')
        x = np.asarray(d['data'], dtype=np.float32).reshape(-1, 3, 32, 32) / 255.0
        y = d['labels'] if 'labels' in d else d['fine_labels']
        return x, np.asarray(y)
    if num_class == 10:
        parts = [_load('data_batch_%d' % i) for i in range(1, 6)]
        xtr = np.concatenate([p[0] for p in parts])
        ytr = np.concatenate([p[1] for p in parts])
        xte, yte = _load('test_batch')
    else:
        xtr, ytr = _load('train')
        xte, yte = _load('test')
    mean = xtr.mean(axis=(0, 2, 3), keepdims=True)
    std = xtr.std(axis=(0, 2, 3), keepdims=True)
    xtr, xte = (xtr - mean) / std, (xte - mean) / std
    if onehot:
        ytr, yte = _onehot(ytr, num_class), _onehot(yte, num_class)
    return xtr.astype(np.float32), ytr, xte.astype(np.float32), yte


# ---- augmentation (reference data.py: crop, flip, whitening, noise) ----------
def random_crop(x, pad=4, seed=None):
    rng = np.random.RandomState(seed)
    n, c, h, w = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    out = np.empty_like(x)
    for i in range(n):
        a, b = rng.randint(0, 2 * pad + 1, 2)
        out[i] = xp[i, :, a:a + h, b:b + w]
    return out


def random_flip(x, seed=None):
    rng = np.random.RandomState(seed)
    flip = rng.rand(x.shape[0]) < 0.5
    out = x.copy()
    out[flip] = out[flip][..., ::-1]
    return out


def whitening(x):
    mean = x.mean(axis=(1, 2, 3), keepdims=True)
    std = np.maximum(x.std(axis=(1, 2, 3), keepdims=True), 1.0 / np.sqrt(x[0].size))
    return (x - mean) / std


def gaussian_noise(x, sigma=0.05, seed=None):
    rng = np.random.RandomState(seed)
    return x + rng.normal(0, sigma, x.shape).astype(x.dtype)


def synthetic_imagenet(n, batch_dtype=np.float32, seed=0, num_classes=1000, hw=224):
    rng = np.random.RandomState(seed)
    x = rng.standard_normal((n, 3, hw, hw)).astype(batch_dtype)
    y = rng.randint(0, num_classes, size=n)
    return x, _onehot(y, num_classes)


def synthetic_criteo(n, num_dense=13, num_sparse=26, vocab=33762577, seed=0):
    """Criteo-shaped synthetic CTR data: dense [n,13] float, sparse [n,26] int64
    ids (global ids across fields, Zipf-skewed), labels [n,1]."""
    rng = np.random.RandomState(seed)
    dense = rng.standard_normal((n, num_dense)).astype(np.float32)
    per = vocab // num_sparse
    z = rng.zipf(1.2, size=(n, num_sparse)) % per
    sparse = (z + np.arange(num_sparse) * per).astype(np.int64)
    y = (rng.rand(n, 1) < 0.25).astype(np.float32)
    return dense, sparse, y
