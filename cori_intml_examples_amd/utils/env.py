"""Environment knobs (device pinning, seeds).

Reference counterpart: the thread/env configuration of ``setup.sh:10-14`` and
``mlextras.configure_session`` (``mlextras.py:35-43``).  On MI355X the relevant
knobs are device pinning (HIP_VISIBLE_DEVICES / LOCAL_RANK) and kernel switches.
"""
from __future__ import annotations

import os
import random

import torch

_GLOBAL_SEED = None


def env_flag(name: str, default: bool) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v.strip().lower() not in ("0", "false", "no", "off", "")


def default_device() -> torch.device:
    """``INTML_DEVICE`` overrides; otherwise the GPU of this process (local rank) if
    one is visible, else the CPU reference backend."""
    dev = os.environ.get("INTML_DEVICE")
    if dev:
        return torch.device(dev)
    if torch.cuda.is_available():
        idx = int(os.environ.get("LOCAL_RANK", "0"))
        n = torch.cuda.device_count()
        return torch.device("cuda", idx % max(n, 1))
    return torch.device("cpu")


def set_random_seed(seed: int) -> None:
    global _GLOBAL_SEED
    _GLOBAL_SEED = int(seed)
    random.seed(seed)
    import numpy as np
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)


def next_seed() -> int:
    """Seed for a new model: derived from the global seed if set, else random."""
    global _GLOBAL_SEED
    if _GLOBAL_SEED is not None:
        _GLOBAL_SEED = (_GLOBAL_SEED * 6364136223846793005 + 1442695040888963407) & 0xFFFFFFFFFFFF
        return _GLOBAL_SEED
    return random.getrandbits(48)
