"""Horovod-keras callbacks (``rpv.py:83-93``; ``DistTrain_mnist.ipynb:494``)."""
from __future__ import annotations

import numpy as np

from ..optim import get_value, set_value
from ..train.callbacks import Callback
from . import dist


class BroadcastGlobalVariablesCallback(Callback):
    """Broadcast weights + optimizer state + iteration counter from ``root_rank``.

    Fires at train begin, i.e. BEFORE the first update (the reference's Horovod
    version broadcasts after batch 0, so its step 0 ran on divergent inits)."""
    needs_batch_logs = False

    def __init__(self, root_rank=0, device=""):
        super().__init__()
        self.root_rank = root_rank
        self.done = False

    def on_train_begin(self, logs=None):
        if self.done:
            return
        dist.broadcast_model_state(self.model, self.root_rank)
        self.done = True


class MetricAverageCallback(Callback):
    """Average every epoch-end log value across ranks with ONE packed all-reduce (R3)."""
    needs_batch_logs = False

    def __init__(self, device=""):
        super().__init__()

    def on_epoch_end(self, epoch, logs=None):
        if logs is None or not logs:
            return
        keys = sorted(k for k, v in logs.items() if np.isscalar(v))
        vals = np.array([float(logs[k]) for k in keys], dtype=np.float64)
        avg = dist.allreduce(vals, average=True)
        for k, v in zip(keys, np.atleast_1d(avg)):
            logs[k] = float(v)


class LearningRateScheduleCallback(Callback):
    needs_batch_logs = False

    def __init__(self, multiplier, start_epoch=0, end_epoch=None, staircase=True,
                 momentum_correction=True, steps_per_epoch=None):
        super().__init__()
        self.start_epoch, self.end_epoch = start_epoch, end_epoch
        self.staircase = staircase
        self.steps_per_epoch = steps_per_epoch
        self.current_epoch = None
        self.initial_lr = None
        self.multiplier = multiplier if callable(multiplier) else (lambda epoch: multiplier)

    def _autodetect_steps_per_epoch(self):
        if self.params.get("steps"):
            return self.params["steps"]
        if self.params.get("samples") and self.params.get("batch_size"):
            return -(-self.params["samples"] // self.params["batch_size"])
        raise ValueError("Could not autodetect the number of steps per epoch.")

    def _adjust(self, epoch):
        set_value(self.model.optimizer.lr, self.initial_lr * self.multiplier(epoch))

    def on_train_begin(self, logs=None):
        self.initial_lr = float(get_value(self.model.optimizer.lr))
        if not self.staircase and not self.steps_per_epoch:
            self.steps_per_epoch = self._autodetect_steps_per_epoch()

    def on_epoch_begin(self, epoch, logs=None):
        self.current_epoch = epoch

    def on_batch_begin(self, batch, logs=None):
        if self.current_epoch < self.start_epoch or (
                self.end_epoch is not None and self.current_epoch >= self.end_epoch):
            return
        if self.staircase and batch == 0:
            self._adjust(self.current_epoch)
        elif not self.staircase:
            self._adjust(self.current_epoch + float(batch) / self.steps_per_epoch)

    def on_epoch_end(self, epoch, logs=None):
        if logs is not None:
            logs["lr"] = float(get_value(self.model.optimizer.lr))


class LearningRateWarmupCallback(LearningRateScheduleCallback):
    """Goyal et al. gradual warmup: lr/size -> lr over ``warmup_epochs`` (``rpv.py:89-92``).
    With warmup_epochs=0 (the reference default) it is a no-op."""

    def __init__(self, warmup_epochs=5, momentum_correction=True, steps_per_epoch=None, verbose=0):
        def multiplier(epoch):
            epoch += 1.0 / self.steps_per_epoch
            return 1.0 / dist.size() * (epoch * (dist.size() - 1) / warmup_epochs + 1)
        super().__init__(multiplier, start_epoch=0, end_epoch=warmup_epochs, staircase=False,
                         momentum_correction=momentum_correction, steps_per_epoch=steps_per_epoch)
        self.verbose = verbose
        self.warmup_epochs = warmup_epochs

    def on_batch_begin(self, batch, logs=None):
        if self.warmup_epochs <= 0:
            return
        super().on_batch_begin(batch, logs)

    def on_epoch_end(self, epoch, logs=None):
        if self.warmup_epochs > 0:
            super().on_epoch_end(epoch, logs)
            if epoch == self.end_epoch - 1 and self.verbose > 0:
                print("\nEpoch %d: finished gradual learning rate warmup to %g." %
                      (epoch + 1, float(get_value(self.model.optimizer.lr))))
