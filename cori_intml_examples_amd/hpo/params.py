"""Hyper-parameter space of the Cray-HPO-style optimizers (``hpo.Params``,
``CrayHPO_rpv.ipynb:99-107``, ``CrayHPO_mnist.ipynb:41-45``).

Each entry is ``[flag, default, domain]``: a tuple ``(lo, hi)`` is a continuous range
(integer when both bounds and the default are ints), a list is a categorical set.
Individuals are dicts ``{flag: value}`` and become command-line arguments
``--h1 16 --dropout 0.2 ...`` for the evaluator command.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Sequence

import numpy as np


class _Dim:
    def __init__(self, flag: str, default, domain):
        self.flag, self.default = flag, default
        if isinstance(domain, tuple):
            if len(domain) != 2:
                raise ValueError("%s: range must be (lo, hi)" % flag)
            lo, hi = domain
            self.kind = "int" if all(isinstance(v, (int, np.integer)) and not isinstance(v, bool)
                                     for v in (lo, hi, default)) else "float"
            self.lo, self.hi = (int(lo), int(hi)) if self.kind == "int" else (float(lo), float(hi))
            if not self.lo <= default <= self.hi:
                raise ValueError("%s: default %r outside %r" % (flag, default, domain))
        elif isinstance(domain, list):
            if not domain:
                raise ValueError("%s: empty choice list" % flag)
            self.kind, self.choices = "cat", list(domain)
        else:
            raise TypeError("%s: domain must be a (lo, hi) tuple or a list" % flag)

    def sample(self, rng: np.random.RandomState):
        if self.kind == "cat":
            return self.choices[rng.randint(len(self.choices))]
        if self.kind == "int":
            return int(rng.randint(self.lo, self.hi + 1))
        return float(rng.uniform(self.lo, self.hi))

    def perturb(self, v, rng: np.random.RandomState, scale: float):
        """Gaussian step of ``scale`` x range width (ints rounded, clipped); categorical
        values are resampled."""
        if self.kind == "cat":
            return self.choices[rng.randint(len(self.choices))]
        width = self.hi - self.lo
        nv = v + rng.normal(0.0, scale * width)
        nv = min(max(nv, self.lo), self.hi)
        return int(round(nv)) if self.kind == "int" else float(nv)


class Params:
    def __init__(self, spec: Sequence[Sequence[Any]]):
        self.dims: List[_Dim] = [_Dim(f, d, dom) for f, d, dom in spec]
        flags = [d.flag for d in self.dims]
        if len(set(flags)) != len(flags):
            raise ValueError("duplicate flags")

    @property
    def flags(self) -> List[str]:
        return [d.flag for d in self.dims]

    def defaults(self) -> Dict[str, Any]:
        return {d.flag: d.default for d in self.dims}

    def sample(self, rng: np.random.RandomState) -> Dict[str, Any]:
        return {d.flag: d.sample(rng) for d in self.dims}

    def mutate(self, ind: Dict[str, Any], rng: np.random.RandomState, rate: float, scale: float = 0.1):
        """Each gene mutates with probability ``rate``."""
        return {d.flag: (d.perturb(ind[d.flag], rng, scale) if rng.rand() < rate else ind[d.flag])
                for d in self.dims}

    def crossover(self, a: Dict[str, Any], b: Dict[str, Any], rng: np.random.RandomState):
        """Uniform crossover."""
        return {d.flag: (a[d.flag] if rng.rand() < 0.5 else b[d.flag]) for d in self.dims}

    @staticmethod
    def format_value(v) -> str:
        if isinstance(v, float):
            if math.isfinite(v) and v == int(v) and abs(v) < 1e15 and not (0 < abs(v) < 1e-4):
                return repr(float(v))
            return "%.6g" % v
        return str(v)

    def to_args(self, ind: Dict[str, Any]) -> List[str]:
        out = []
        for d in self.dims:
            out += [d.flag, self.format_value(ind[d.flag])]
        return out

    def __len__(self):
        return len(self.dims)

    def __repr__(self):
        return "Params(%s)" % ", ".join(d.flag for d in self.dims)
