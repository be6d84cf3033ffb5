"""Counter-based RNG shared bit-for-bit by the HIP kernels and the CPU reference.

Dropout masks are never stored: every kernel that needs a keep/drop decision
recomputes it from ``(seed, stream, step, logical element index)``.  The same
hash lives in ``csrc/kernels/common.h`` (``rng_u32``); this file is its torch
twin so CPU tests and the CPU plumbing backend see identical masks.

Reference: Keras ``Dropout`` (``mnist.py:52,55``, ``rpv.py:50,56``) draws a fresh
mask every batch with TF's stateful RNG; we use a stateless hash instead so the
backward pass (and HIP-graph replays) can regenerate the mask.
"""
from __future__ import annotations

import torch

_M32 = 0xFFFFFFFF
GOLDEN = 0x9E3779B9
MIX2 = 0x85EBCA6B


def _fmix32(x: torch.Tensor) -> torch.Tensor:
    # murmur3 finaliser on int64 tensors holding uint32 values
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & _M32
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & _M32
    x = x ^ (x >> 16)
    return x


def rng_u32(idx: torch.Tensor, seed: int, stream: int, step: int) -> torch.Tensor:
    """uint32 hash (as int64) of element indices ``idx`` (int64 tensor)."""
    x = (idx & _M32) ^ ((step * GOLDEN) & _M32)
    x = _fmix32(x ^ (seed & _M32))
    x = _fmix32((x + ((stream * MIX2) & _M32)) & _M32)
    return x


def keep_threshold(rate: float) -> int:
    """24-bit threshold: element kept iff (u >> 8) >= thr."""
    return min(int(rate * 16777216.0), 16777216)


def dropout_keep(numel: int, rate: float, seed: int, stream: int, step: int,
                 device="cpu") -> torch.Tensor:
    """Bool keep-mask over a logical flat index range [0, numel)."""
    idx = torch.arange(numel, dtype=torch.int64, device=device)
    u = rng_u32(idx, seed, stream, step)
    return (u >> 8) >= keep_threshold(rate)


def uniform01(numel: int, seed: int, stream: int, step: int = 0, device="cpu") -> torch.Tensor:
    idx = torch.arange(numel, dtype=torch.int64, device=device)
    u = rng_u32(idx, seed, stream, step)
    return (u >> 8).to(torch.float32) * (1.0 / 16777216.0)


def u01_of(u: torch.Tensor) -> torch.Tensor:
    """fp32 in [0, 1) from hash values (int64 holding uint32): (u >> 8) * 2^-24, exact."""
    return (u >> 8).to(torch.float32) * torch.tensor(2.0 ** -24, dtype=torch.float32)


def uint_below(u: torch.Tensor, m: int) -> torch.Tensor:
    """floor((u >> 8) * m / 2^24): an integer in [0, m) (csrc/kernels/synth.hip uint_below)."""
    return ((u >> 8) * m) >> 24


def init_uniform(numel: int, scale: float, seed: int, stream: int) -> torch.Tensor:
    """uniform(-scale, scale) of a parameter span: (u01 * 2 - 1) * scale in fp32, each op
    rounded once -- bit-identical to init_params_kernel (csrc/kernels/synth.hip)."""
    idx = torch.arange(numel, dtype=torch.int64)
    u = u01_of(rng_u32(idx, seed & _M32, stream & _M32, 0))
    return (u * torch.tensor(2.0, dtype=torch.float32) - torch.tensor(1.0, dtype=torch.float32)) * \
        torch.tensor(scale, dtype=torch.float32)
