"""Synthetic data sets on the counter-based RNG.

``synth_device`` fills a device-resident data set with ``synth_kernel``
(``csrc/kernels/synth.hip``) where the model trains -- no host generation, no upload;
``synth_cpu`` is its bit-identical torch twin (the same single-rounded fp32 operations, in
the same order, on the same hash integers), so CPU reference runs and tests see exactly
the samples the GPU trains on.  Sample ``i`` depends only on ``(seed, i)``: a rank or an
HPO engine can generate its own shard ``[first, first + n)``.

Kinds (the reference trains on RPV HDF5 files / MNIST downloads this image does not have):

* ``uniform`` -- pixels u01, labels from the hash (the bench's throughput data);
* ``rpv`` -- calorimeter-like images: 2-3 wide "jets" (background) or 4-6 narrow ones
  (signal, label 1) as separable quadratic bumps on uniform noise (cf. io/datasets.synthetic_rpv);
* ``mnist`` -- 10 class templates (thresholded hash, smoothed with the pixels above and to
  the left), translated by -3..3 pixels per sample, plus uniform noise of amplitude 0.5,
  clipped to [0, 1] (cf. io/datasets.synthetic_mnist).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from ..ops.rng import rng_u32, u01_of, uint_below

KINDS = {"uniform": 0, "rpv": 1, "mnist": 2}
S_LAB, S_NJ, S_CY, S_CX, S_AMP, S_CH, S_NOISE, S_TPL, S_MCLS, S_MNOISE, S_SHIFT = range(1, 12)
_M32 = 0xFFFFFFFF
RPV_JETS = 6


def _f(v) -> torch.Tensor:
    return torch.tensor(np.float32(v), dtype=torch.float32)


def _bump(d: torch.Tensor, r2inv: torch.Tensor) -> torch.Tensor:
    t = torch.clamp_min(_f(1.0) - (d * d).to(torch.float32) * r2inv, 0.0)
    return t * t


def synth_cpu(kind: str, n: int, shape: Tuple[int, int, int], ncls: int, seed: int,
              first: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Samples [first, first + n): x fp32 [n, H, W, C] (round to bf16 for the device values),
    y fp32 [n, ncls]."""
    H, W, C = shape
    k = KINDS[kind]
    seed &= _M32
    i = torch.arange(first, first + n, dtype=torch.int64) & _M32
    yy = torch.arange(H, dtype=torch.int64)
    xx = torch.arange(W, dtype=torch.int64)
    cc = torch.arange(C, dtype=torch.int64)
    pix = ((((i[:, None, None, None] * H + yy[None, :, None, None]) & _M32) * W + xx[None, None, :, None]) & _M32)
    pix = ((pix * C) & _M32) + cc[None, None, None, :]
    pix = pix & _M32
    if k == 1:
        ul = rng_u32(i, seed, S_LAB, 0)
        sig = (ul >> 8) < (1 << 23)
        cls = sig.to(torch.int64)
        un = rng_u32(i, seed, S_NJ, 0)
        nj = torch.where(sig, 4 + uint_below(un, 3), 2 + uint_below(un, 2))
        r2inv = torch.where(sig, _f(1.0) / _f(9.0), _f(1.0) / _f(36.0))[:, None]
        v = torch.zeros(n, H, W, C, dtype=torch.float32)
        for j in range(RPV_JETS):
            kk = (i * 8 + j) & _M32
            jy = uint_below(rng_u32(kk, seed, S_CY, 0), H)
            jx = uint_below(rng_u32(kk, seed, S_CX, 0), W)
            jc = uint_below(rng_u32(kk, seed, S_CH, 0), C)
            amp = _f(0.5) + _f(2.0) * u01_of(rng_u32(kk, seed, S_AMP, 0))
            amp = torch.where(j < nj, amp, _f(0.0))
            gy = _bump(yy[None, :] - jy[:, None], r2inv)                   # [n, H]
            gx = _bump(xx[None, :] - jx[:, None], r2inv)                   # [n, W]
            term = (amp[:, None] * gy)[:, :, None] * gx[:, None, :]        # [n, H, W]
            on = (jc[:, None] == cc[None, :])                               # [n, C]
            v = torch.where(on[:, None, None, :], v + term[..., None], v)
        v = v + _f(0.05) * u01_of(rng_u32(pix, seed, S_NOISE, 0))
    elif k == 2:
        cls = uint_below(rng_u32(i, seed, S_MCLS, 0), ncls)
        t = torch.arange(ncls * H * W, dtype=torch.int64)
        tpl = ((rng_u32(t, seed, S_TPL, 0) >> 8) >= 11744051).to(torch.float32).view(ncls, H, W)
        sm = ((tpl + torch.roll(tpl, 1, 1)) + torch.roll(tpl, 1, 2)) * (_f(1.0) / _f(3.0))
        us = rng_u32(i, seed, S_SHIFT, 0)
        sy, sx = uint_below(us, 7) - 3, (us & 0xFF) % 7 - 3             # per-sample translation
        ty = (yy[None, :] - sy[:, None]) % H                             # [n, H]
        tx = (xx[None, :] - sx[:, None]) % W                             # [n, W]
        img = sm[cls[:, None, None], ty[:, :, None], tx[:, None, :]]     # [n, H, W]
        noise = _f(0.5) * (_f(2.0) * u01_of(rng_u32(pix, seed, S_MNOISE, 0)) - _f(1.0))
        v = torch.clamp(img[..., None] + noise, 0.0, 1.0)
    else:
        ul = rng_u32(i, seed, S_LAB, 0)
        cls = (u01_of(ul) < _f(0.5)).to(torch.int64) if ncls == 1 else uint_below(ul, ncls)
        v = u01_of(rng_u32(pix, seed, S_NOISE, 0))
    if ncls == 1:
        y = cls.to(torch.float32)[:, None]
    else:
        y = torch.nn.functional.one_hot(cls, ncls).to(torch.float32)
    return v, y


def synth_device(kind: str, n: int, shape: Tuple[int, int, int], ncls: int, Cs: int, seed: int,
                 device, first: int = 0):
    """A device-resident data set (executor_base.DeviceData: x bf16 [n, H*W*Cs] with the
    channel padding zeroed, y fp32 [n, ncls]) generated on the GPU by synth_kernel."""
    from ..models.executor_base import DeviceData
    from ..ops import hip
    H, W, C = shape
    dev = torch.device(device)
    x = torch.empty(n, H * W * Cs, dtype=torch.bfloat16, device=dev)
    y = torch.empty(n, ncls, dtype=torch.float32, device=dev)
    if dev.type != "cuda":
        v, yt = synth_cpu(kind, n, shape, ncls, seed, first)
        xs = torch.zeros(n, H, W, Cs, dtype=torch.bfloat16)
        xs[..., :C] = v.to(torch.bfloat16)
        return DeviceData(xs.reshape(n, -1).to(dev), yt.to(dev), n)
    K = hip.kernels()
    a = K.SynthArgs()
    a.x, a.y = x.data_ptr(), y.data_ptr()
    a.n, a.first, a.H, a.W, a.C, a.Cs, a.ncls, a.kind = n, first, H, W, C, Cs, ncls, KINDS[kind]
    a.seed = seed & _M32
    K.synth(a, hip.stream_handle())
    return DeviceData(x, y, n)


def for_model(model, kind: str, n: int, seed: int, first: int = 0):
    """A synthetic data set in ``model``'s executor layout, generated where it trains: on the
    GPU by synth_kernel for the HIP executor, by the CPU twin (bf16-rounded, so both see the
    same pixel values) for the CPU reference executor.  ``Model.fit`` / ``evaluate`` accept
    the returned DeviceData in place of (x, y) arrays."""
    ex = model._executor
    plan = ex.plan
    shape = tuple(plan.input_shape)
    ncls = plan.head.N
    if hasattr(ex, "in_Cs") and torch.device(ex.device).type == "cuda":
        return synth_device(kind, n, shape, ncls, ex.in_Cs, seed, ex.device, first)
    v, y = synth_cpu(kind, n, shape, ncls, seed, first)
    return ex.upload(v.to(torch.bfloat16).float().numpy(), y.numpy())


def split(data, frac: float):
    """Keras ``validation_split`` on a DeviceData: the LAST ``frac`` of the samples is the
    validation set (views, no copy)."""
    from ..models.executor_base import DeviceData
    s = int(data.n * (1.0 - frac))
    return (DeviceData(data.x[:s], data.y[:s], s), DeviceData(data.x[s:], data.y[s:], data.n - s))


S_FLIP, S_RELABEL = 12, 13


def flip_labels(data, frac: float, seed: int, first: int = 0):
    """Label noise in place: each sample ``i`` (counted from ``first``) keeps its label unless
    ``u01(rng(i, seed)) < frac``; a flipped binary label becomes ``1 - y``, a flipped one-hot
    class moves to a uniformly drawn OTHER class.  Pure integer hashing (ops/rng), so the
    device and CPU data sets agree bit for bit.  Makes the synthetic tasks non-separable: the
    best trial of an HPO sits above the ~H(frac) noise floor instead of at 1e-5, so choosing
    it means something (tests/test_convergence.py uses the same 10 %)."""
    if frac <= 0:
        return data
    y = data.y
    dev = y.device
    i = (torch.arange(first, first + data.n, dtype=torch.int64, device=dev)) & _M32
    flip = u01_of(rng_u32(i, seed & _M32, S_FLIP, 0)) < _f(frac).to(dev)
    ncls = y.shape[1]
    if ncls == 1:
        y[:, 0] = torch.where(flip, 1.0 - y[:, 0], y[:, 0])
    else:
        cls = y.argmax(1)
        new = (cls + 1 + uint_below(rng_u32(i, seed & _M32, S_RELABEL, 0), ncls - 1)) % ncls
        cls = torch.where(flip, new, cls)
        y.copy_(torch.nn.functional.one_hot(cls, ncls).to(y.dtype))
    return data
