"""MNIST recipe (``mnist.py:1-59``): constants, ``load_data`` and ``build_model``, used by
the MNIST HPO notebooks (``DistHPO_mnist.ipynb:37,174``, ``HPO_mnist.ipynb:44``,
``DistWidgetHPO_mnist.ipynb:42,183``).

``load_data`` reads the Keras cache file ``~/.keras/datasets/mnist.npz`` (or
``$INTML_MNIST_NPZ``) when present -- there is no network to download it -- and otherwise
returns a learnable synthetic MNIST of the same shapes/dtypes.
"""
from __future__ import annotations

import os
import warnings

import numpy as np

from ..io.datasets import synthetic_mnist
from ..utils import to_categorical
from .zoo import mnist_cnn

n_classes = 10
img_rows, img_cols = 28, 28


def _npz_path():
    p = os.environ.get("INTML_MNIST_NPZ")
    if p:
        return p
    return os.path.join(os.path.expanduser("~"), ".keras", "datasets", "mnist.npz")


def load_data(synthetic_ok: bool = True, n_train: int = 60000, n_test: int = 10000):
    """``(x_train, y_train, x_test, y_test)``: float32 NHWC in [0, 1], one-hot labels
    (``mnist.py:32-42``)."""
    p = _npz_path()
    if os.path.exists(p):
        with np.load(p, allow_pickle=False) as f:
            xtr, ytr, xte, yte = f["x_train"], f["y_train"], f["x_test"], f["y_test"]
        shape = (img_rows, img_cols, 1)
        xtr = xtr.reshape((xtr.shape[0],) + shape).astype(np.float32) / 255
        xte = xte.reshape((xte.shape[0],) + shape).astype(np.float32) / 255
        return xtr, to_categorical(ytr, n_classes), xte, to_categorical(yte, n_classes)
    if not synthetic_ok:
        raise FileNotFoundError(p)
    warnings.warn("MNIST cache %s not found (no network): using synthetic MNIST-shaped data" % p)
    return synthetic_mnist(n_train, n_test)


def build_model(h1=4, h2=8, h3=32, dropout=0.5, optimizer="Adadelta", device=None, use_horovod=False):
    """Sequential CNN of ``mnist.py:44-59`` compiled with CCE + accuracy."""
    return mnist_cnn(h1=h1, h2=h2, h3=h3, dropout=dropout, optimizer=optimizer, n_classes=n_classes,
                     input_shape=(img_rows, img_cols, 1), use_horovod=use_horovod, device=device)
