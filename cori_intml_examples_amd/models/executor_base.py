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


class Executor:
    """Runs training / evaluation steps of a compiled Plan on one device."""

    device: torch.device

    def __init__(self, plan: Plan, store, optimizer, seed: int):
        self.plan = plan
        self.store = store
        self.optimizer = optimizer
        self.seed = int(seed) & 0xFFFFFFFF
        self.reducer = None          # data-parallel gradient reducer (parallel.dist)

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
