"""Datasets: synthetic stand-ins with the reference's shapes, and the RPV HDF5 loader.

There is no network here (the reference downloads MNIST via ``keras.datasets``,
``mnist.py:35``, and reads RPV HDF5 files from Cori scratch, ``rpv.py:19-36``), so
benchmarks and tests use synthetic data of the same shape/dtype.  The generators are
*learnable* (class-conditional templates + noise) so loss curves behave like real
training, which HPO tests rely on.
"""
from __future__ import annotations

import os
from typing import Tuple

import numpy as np


def synthetic_mnist(n_train: int = 60000, n_test: int = 10000, seed: int = 0, n_classes: int = 10,
                    rows: int = 28, cols: int = 28, noise: float = 0.35):
    """Returns (x_train, y_train_onehot, x_test, y_test_onehot); float32 NHWC in [0,1]."""
    rng = np.random.RandomState(seed)
    templates = (rng.rand(n_classes, rows, cols) > 0.7).astype(np.float32)
    # smooth templates a bit so conv features matter
    t = templates
    t = (t + np.roll(t, 1, 1) + np.roll(t, 1, 2)) / 3.0

    def make(n, rs):
        lab = rs.randint(0, n_classes, size=n)
        x = t[lab] + noise * rs.randn(n, rows, cols).astype(np.float32)
        x = np.clip(x, 0.0, 1.0).astype(np.float32)[..., None]
        y = np.zeros((n, n_classes), np.float32)
        y[np.arange(n), lab] = 1.0
        return x, y

    xtr, ytr = make(n_train, np.random.RandomState(seed + 1))
    xte, yte = make(n_test, np.random.RandomState(seed + 2))
    return xtr, ytr, xte, yte


def synthetic_rpv(n: int, channels: int = 1, size: int = 64, seed: int = 0, signal_frac: float = 0.5,
                  chunk: int = 4096):
    """Synthetic calorimeter images: background = diffuse noise + 2-3 wide jets, signal =
    4-6 narrower jets (an RPV gluino decay has more jets).  Jets are separable Gaussians,
    generated vectorised in chunks (~1 s per 100k 64x64 images).  Returns
    (hist [n,size,size,C] float32, y [n] float32, weight [n] float32)."""
    rs = np.random.RandomState(seed)
    y = (rs.rand(n) < signal_frac).astype(np.float32)
    weight = (0.5 + rs.rand(n)).astype(np.float32)
    x = np.empty((n, size, size, channels), np.float32)
    J = 6
    grid = np.arange(size, dtype=np.float32)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        m = hi - lo
        sig = y[lo:hi] > 0
        njets = np.where(sig, rs.randint(4, 7, size=m), rs.randint(2, 4, size=m))
        cy = rs.randint(0, size, size=(m, J)).astype(np.float32)
        cx = rs.randint(0, size, size=(m, J)).astype(np.float32)
        amp = (rs.rand(m, J) * 2 + 0.5).astype(np.float32) * (np.arange(J)[None, :] < njets[:, None])
        ch = rs.randint(0, channels, size=(m, J))
        w = np.where(sig, 1.5, 3.0).astype(np.float32)[:, None, None]
        gy = np.exp(-((grid[None, None, :] - cy[:, :, None]) ** 2) / (2 * w * w))      # (m, J, size)
        gx = np.exp(-((grid[None, None, :] - cx[:, :, None]) ** 2) / (2 * w * w))
        noise = 0.05 * rs.rand(m, size, size, channels).astype(np.float32)
        for c in range(channels):      # sum_j amp_j [ch_j == c] gy_j (x) gx_j  as one batched GEMM
            a = amp * (ch == c)
            x[lo:hi, :, :, c] = np.matmul((gy * a[:, :, None]).transpose(0, 2, 1), gx) + noise[..., c]
    return x, y, weight


# ----------------------------------------------------------------------------- RPV HDF5
def load_file(filename: str, n_samples: int):
    """Read ``all_events/{hist,y,weight}`` (first n_samples) and add a channel axis
    (``rpv.py:19-25``)."""
    from .h5 import H5File
    with H5File(filename, "r") as f:
        hist = f.read_dataset("all_events/hist", n_samples)
        y = f.read_dataset("all_events/y", n_samples)
        w = f.read_dataset("all_events/weight", n_samples)
    if hist.ndim == 3:
        hist = hist[:, :, :, None]
    return hist.astype(np.float32), y.astype(np.float32), w.astype(np.float32)


def load_dataset(path: str, n_train: int = 412416, n_valid: int = 137471, n_test: int = 137471):
    """``rpv.py:27-36``: train.h5 / val.h5 / test.h5 in ``path``."""
    out = []
    for name, n in (("train.h5", n_train), ("val.h5", n_valid), ("test.h5", n_test)):
        out.append(load_file(os.path.join(path, name), n))
    return tuple(out)


def write_rpv_file(filename: str, hist: np.ndarray, y: np.ndarray, weight: np.ndarray) -> None:
    """Write the RPV schema: group ``all_events`` with datasets
    ``hist`` (N,H,W), ``y`` (N,), ``weight`` (N,)."""
    from .h5 import H5File
    if hist.ndim == 4 and hist.shape[-1] == 1:
        hist = hist[..., 0]
    with H5File(filename, "w") as f:
        f.create_group("all_events")
        f.write_dataset("all_events/hist", np.ascontiguousarray(hist, dtype=np.float32))
        f.write_dataset("all_events/y", np.ascontiguousarray(y, dtype=np.float32))
        f.write_dataset("all_events/weight", np.ascontiguousarray(weight, dtype=np.float32))


def make_synthetic_rpv_dir(path: str, n_train: int, n_valid: int, n_test: int, channels: int = 1,
                           seed: int = 0) -> str:
    os.makedirs(path, exist_ok=True)
    for i, (name, n) in enumerate((("train.h5", n_train), ("val.h5", n_valid), ("test.h5", n_test))):
        x, y, w = synthetic_rpv(n, channels=channels, seed=seed + i)
        if channels == 1:
            write_rpv_file(os.path.join(path, name), x, y, w)
        else:
            from .h5 import H5File
            with H5File(os.path.join(path, name), "w") as f:
                f.create_group("all_events")
                f.write_dataset("all_events/hist", x)
                f.write_dataset("all_events/y", y)
                f.write_dataset("all_events/weight", w)
    return path
