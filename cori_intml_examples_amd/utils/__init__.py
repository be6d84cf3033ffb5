import numpy as np

from .env import default_device, env_flag, set_random_seed


def to_categorical(y, num_classes=None, dtype="float32"):
    """One-hot encode integer class vectors (``keras.utils.to_categorical``, ``mnist.py:40-41``)."""
    y = np.asarray(y, dtype="int64").reshape(-1)
    n = int(num_classes) if num_classes is not None else int(y.max()) + 1
    out = np.zeros((y.shape[0], n), dtype=dtype)
    out[np.arange(y.shape[0]), y] = 1
    return out


__all__ = ["default_device", "env_flag", "set_random_seed", "to_categorical"]
