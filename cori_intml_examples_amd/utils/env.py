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


_TUNE = None


def tune(key: str, default):
    """Kernel-path / geometry tuning value ``key`` (executor switches and launch geometry):
    ``default`` unless ``INTML_TUNE="key=value,key=value"`` overrides it (measurement sweeps
    and A/B tests).  One knob for all of them instead of one environment variable each; the
    value is parsed as the default's type (bool: 0/1/true/false)."""
    global _TUNE
    if _TUNE is None or _TUNE[0] != os.environ.get("INTML_TUNE", ""):
        raw = os.environ.get("INTML_TUNE", "")
        d = {}
        for item in raw.split(","):
            if "=" in item:
                k, v = item.split("=", 1)
                d[k.strip()] = v.strip()
        _TUNE = (raw, d)
    v = _TUNE[1].get(key)
    if v is None:
        return default
    if isinstance(default, bool):
        return v.lower() not in ("0", "false", "no", "off", "")
    if isinstance(default, int):
        return int(v)
    if isinstance(default, float):
        return float(v)
    return v


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
