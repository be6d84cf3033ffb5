"""Executor interface shared by the HIP (gfx950) and CPU-reference backends."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .plan import Plan


@dataclass
class DeviceData:
    """A dataset resident on the executor's device (whole set, uploaded once)."""
    x: torch.Tensor          # executor-specific layout
    y: torch.Tensor          # [N, C] fp32 targets (one-hot for categorical)
    n: int


def prepare_targets(y: np.ndarray, plan: Plan) -> np.ndarray:
    y = np.asarray(y)
    head = plan.head
    if head.loss == "sparse_categorical_crossentropy":
        yi = y.reshape(-1).astype(np.int64)
        out = np.zeros((yi.shape[0], head.N), np.float32)
        out[np.arange(yi.shape[0]), yi] = 1.0
        return out
    y = y.astype(np.float32)
    if y.ndim == 1:
        y = y.reshape(-1, 1)
    if y.shape[1] != head.N:
        raise ValueError("targets have %d columns, model outputs %d" % (y.shape[1], head.N))
    return np.ascontiguousarray(y)


def warmup_lr(g: int, spe: int, size: int, epochs: float, base: float) -> float:
    """LR of 0-based warmup step g: ramps linearly from ~base/size to base over
    ``epochs * spe`` steps (Goyal et al. 2017 gradual warmup; the same schedule the device
    bookkeeping computes, misc.hip step_bookkeeping)."""
    return base / size * ((g + 1) / spe * (size - 1) / epochs + 1.0)


class Executor:
    """Runs training / evaluation steps of a compiled Plan on one device."""

    device: torch.device

    def __init__(self, plan: Plan, store, optimizer, seed: int):
        self.plan = plan
        self.store = store
        self.optimizer = optimizer
        self.seed = int(seed) & 0xFFFFFFFF
        self.reducer = None          # data-parallel gradient reducer (parallel.dist)
        self.lr_warmup = None        # (t0, steps, spe, size, epochs, base) device LR schedule

    # learning-rate schedule ---------------------------------------------------------------
    def set_lr_warmup(self, t0: int, steps: int, spe: int, size: int, epochs: float, base: float) -> None:
        """Gradual LR warmup evaluated per step by the executor itself (no per-batch host
        write): optimizer step g = iterations - t0 - 1 < steps uses
        ``warmup_lr(g, ...)`` as its base LR (``parallel.callbacks.LearningRateWarmupCallback``)."""
        self.lr_warmup = (int(t0), int(steps), int(spe), int(size), float(epochs), float(base)) if steps > 0 else None

    def base_lr_for_step(self, t: int, host_lr: float) -> float:
        """Base LR of optimizer iteration ``t`` (1-based), before Keras ``decay``."""
        w = self.lr_warmup
        if w is not None:
            t0, steps, spe, size, epochs, base = w
            g = t - t0 - 1
            if 0 <= g < steps:
                return warmup_lr(g, spe, size, epochs, base)
        return host_lr

    # data ---------------------------------------------------------------------------------
    def upload(self, x: np.ndarray, y: Optional[np.ndarray]) -> DeviceData:
        raise NotImplementedError

    # steps --------------------------------------------------------------------------------
    def train_step(self, data: DeviceData, perm: torch.Tensor, pos: int, bs: int) -> None:
        raise NotImplementedError

    def train_steps(self, data: DeviceData, perm: torch.Tensor, pos: int, bs: int, k: int) -> None:
        """``k`` consecutive full batches starting at ``pos`` (backends may fuse them)."""
        for i in range(k):
            self.train_step(data, perm, pos + i * bs, bs)

    def eval_step(self, data: DeviceData, pos: int, bs: int) -> None:
        raise NotImplementedError

    def predict_step(self, data: DeviceData, pos: int, bs: int) -> torch.Tensor:
        raise NotImplementedError

    # metrics ------------------------------------------------------------------------------
    def reset_metrics(self) -> None:
        raise NotImplementedError

    def read_metrics(self):
        """(mean_loss, mean_acc, count) since the last reset; synchronises."""
        raise NotImplementedError

    def last_batch_metrics(self):
        raise NotImplementedError

    # params -------------------------------------------------------------------------------
    def params_changed(self) -> None:
        """Called after the host overwrote master weights (set_weights/load/broadcast)."""

    def optimizer_state(self):
        """List of flat fp32 slot tensors (Keras optimizer weights, minus iterations)."""
        raise NotImplementedError

    def set_optimizer_state(self, iterations: int, slots) -> None:
        raise NotImplementedError

    def synchronize(self) -> None:
        pass
