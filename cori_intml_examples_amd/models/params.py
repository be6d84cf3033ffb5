"""Flat parameter / gradient store.

Every trainable tensor of the model lives in ONE contiguous fp32 master buffer in
Keras layer order (kernel, bias per layer) and Keras layout.  Gradients land in
an identically laid-out flat buffer, so data-parallel gradient buckets are plain
views (no flatten/unflatten copies) and the fused optimizer is a single
multi-tensor launch over the whole buffer.  Reference counterpart: the per-
variable gradients Horovod fuses into its fusion buffer (``rpv.py:63-65``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np
import torch

from .layers import Layer


@dataclass
class ParamSpec:
    layer: Layer
    short: str                 # 'kernel' | 'bias'
    shape: Tuple[int, ...]
    init: str
    offset: int
    numel: int

    @property
    def name(self) -> str:
        return "%s/%s:0" % (self.layer.name, self.short)


class ParamStore:
    def __init__(self, layers: List[Layer], device: torch.device):
        self.device = torch.device(device)
        self.specs: List[ParamSpec] = []
        off = 0
        for layer in layers:
            for short, shape, init in layer.weight_specs():
                n = int(np.prod(shape))
                self.specs.append(ParamSpec(layer, short, tuple(shape), init, off, n))
                off += n
        self.numel = off
        # keep the buffer size a multiple of 64 floats so vectorised kernels need no tails
        self.capacity = max(64, (off + 63) // 64 * 64)
        self.master = torch.zeros(self.capacity, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.capacity, dtype=torch.float32, device=self.device)
        self._bind_views()

    def _bind_views(self):
        for s in self.specs:
            s.layer._weights[s.short] = self.master[s.offset:s.offset + s.numel].view(s.shape)

    def spec(self, layer: Layer, short: str) -> ParamSpec:
        for s in self.specs:
            if s.layer is layer and s.short == short:
                return s
        raise KeyError((layer.name, short))

    def view(self, layer: Layer, short: str, grad: bool = False) -> torch.Tensor:
        s = self.spec(layer, short)
        buf = self.grad if grad else self.master
        return buf[s.offset:s.offset + s.numel].view(s.shape)

    def has(self, layer: Layer, short: str) -> bool:
        return any(s.layer is layer and s.short == short for s in self.specs)

    # -- initialisation (Keras defaults: glorot_uniform kernels, zero biases) -------------
    def initialize(self, seed: int) -> None:
        """Keras initialisers.  Uniform kinds (glorot / he uniform) and constants run on the
        counter-based RNG -- the init kernel on a GPU (K16, csrc/kernels/synth.hip), its
        bit-identical torch twin on the CPU (ops/rng.init_uniform) -- so the same seed gives
        the same weights on both backends with no host round trip; the parameter index is
        the RNG stream.  Normal kinds are drawn on the host."""
        from ..ops import rng
        on_gpu = self.device.type == "cuda"
        K = None
        if on_gpu:
            from ..ops import hip
            K = hip.kernels()
        g = torch.Generator().manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
        host = None
        for idx, s in enumerate(self.specs):
            init = s.init if isinstance(s.init, str) else "glorot_uniform"
            if len(s.shape) == 4:
                rf = s.shape[0] * s.shape[1]
                fan_in, fan_out = s.shape[2] * rf, s.shape[3] * rf
            elif len(s.shape) == 2:
                fan_in, fan_out = s.shape
            else:
                fan_in = fan_out = s.numel
            kind, scale = None, 0.0
            if init in ("zeros", "Zeros"):
                kind = 0
            elif init in ("ones", "Ones"):
                kind = 1
            elif init in ("glorot_uniform", "VarianceScaling"):
                kind, scale = 2, math.sqrt(6.0 / (fan_in + fan_out))
            elif init == "he_uniform":
                kind, scale = 2, math.sqrt(6.0 / fan_in)
            elif init == "glorot_normal":
                std = math.sqrt(2.0 / (fan_in + fan_out))
                vals = torch.randn(s.numel, generator=g) * std
                self.master[s.offset:s.offset + s.numel].copy_(vals.to(self.device))
                continue
            else:
                raise NotImplementedError("initializer %s" % init)
            if on_gpu:
                a = K.InitArgs()
                a.p = self.master.data_ptr() + 4 * s.offset
                a.n, a.kind, a.scale, a.seed, a.stream = s.numel, kind, float(scale), int(seed) & 0xFFFFFFFF, idx
                K.init_params(a, hip.stream_handle())
            else:
                if host is None:
                    host = self.master.detach()
                seg = host[s.offset:s.offset + s.numel]
                if kind == 2:
                    seg.copy_(rng.init_uniform(s.numel, scale, int(seed), idx))
                else:
                    seg.fill_(float(kind))

    # -- host I/O --------------------------------------------------------------------------
    def get_weights(self) -> List[np.ndarray]:
        host = self.master.detach().cpu()
        return [host[s.offset:s.offset + s.numel].view(s.shape).numpy().copy() for s in self.specs]

    def set_weights(self, values) -> None:
        if len(values) != len(self.specs):
            raise ValueError("expected %d arrays, got %d" % (len(self.specs), len(values)))
        host = self.master.detach().cpu().clone()
        for s, v in zip(self.specs, values):
            t = torch.as_tensor(np.asarray(v), dtype=torch.float32)
            if tuple(t.shape) != s.shape:
                raise ValueError("%s: shape %s != %s" % (s.name, tuple(t.shape), s.shape))
            host[s.offset:s.offset + s.numel] = t.reshape(-1)
        self.master.copy_(host.to(self.device))

    def layer_ranges(self) -> Dict[str, Tuple[int, int]]:
        out: Dict[str, Tuple[int, int]] = {}
        for s in self.specs:
            lo, hi = out.get(s.layer.name, (s.offset, s.offset))
            out[s.layer.name] = (min(lo, s.offset), max(hi, s.offset + s.numel))
        return out
