"""Keras-named loss functions (``keras.losses``; ``mnist.py:58`` passes
``categorical_crossentropy`` as a function).  ``compile`` recognises them by name and runs
the fused HIP loss head; calling them directly evaluates the Keras 2.2 formula (clipped
probabilities, per-sample loss) on numpy / torch inputs."""
from __future__ import annotations

import numpy as np

EPSILON = 1e-7


def _np(x):
    try:
        import torch
        if isinstance(x, torch.Tensor):
            return x.detach().cpu().double().numpy()
    except ImportError:
        pass
    return np.asarray(x, dtype=np.float64)


def categorical_crossentropy(y_true, y_pred):
    yt, yp = _np(y_true), _np(y_pred)
    yp = yp / yp.sum(axis=-1, keepdims=True)
    yp = np.clip(yp, EPSILON, 1 - EPSILON)
    return -(yt * np.log(yp)).sum(axis=-1)


def binary_crossentropy(y_true, y_pred):
    yt, yp = _np(y_true), np.clip(_np(y_pred), EPSILON, 1 - EPSILON)
    logits = np.log(yp / (1 - yp))
    per = np.maximum(logits, 0) - logits * yt + np.log1p(np.exp(-np.abs(logits)))
    return per.mean(axis=-1)


def mean_squared_error(y_true, y_pred):
    return ((_np(y_pred) - _np(y_true)) ** 2).mean(axis=-1)


def sparse_categorical_crossentropy(y_true, y_pred):
    yp = _np(y_pred)
    yt = _np(y_true).astype(np.int64).reshape(-1)
    onehot = np.zeros_like(yp)
    onehot[np.arange(len(yt)), yt] = 1
    return categorical_crossentropy(onehot, yp)


mse = MSE = mean_squared_error


def get(identifier):
    if callable(identifier):
        return identifier
    return globals()[identifier]
