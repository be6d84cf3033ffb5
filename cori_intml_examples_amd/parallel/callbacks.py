"""Horovod-keras callbacks (``rpv.py:83-93``; ``DistTrain_mnist.ipynb:494``).

Attribution: ``LearningRateScheduleCallback`` / ``LearningRateWarmupCallback`` follow the
semantics (steps-per-epoch autodetection, the Goyal et al. 2017 warmup multiplier, messages)
of Horovod's Keras callbacks of the same names (Horovod, Apache License 2.0, Copyright 2018
Uber Technologies, Inc.); the schedule itself runs on the device (``StepState`` warmup
fields, ``misc.hip`` step bookkeeping), not in a per-batch host callback.
"""
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
    """Generic per-epoch (staircase) or per-batch LR multiplier schedule, host-driven.

    Same constructor and semantics as ``horovod.keras.callbacks.LearningRateScheduleCallback``
    (Apache-2.0, Uber Technologies; API shape and behaviour followed for drop-in use, not
    its code).  A non-staircase schedule writes the LR every batch and so forces the fit
    loop to one step per graph replay; the warmup below avoids that."""
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


class LearningRateWarmupCallback(Callback):
    """Gradual LR warmup from ``lr / size`` to ``lr`` over ``warmup_epochs`` (Goyal et al.
    2017; the schedule ``rpv.py:89-92`` requests through Horovod's callback of this name).

    The ramp is evaluated BY THE EXECUTOR for every optimizer step (device step bookkeeping
    on the GPU, ``misc.hip:step_bookkeeping``): this callback only registers it at train
    begin, so it neither writes the LR per batch nor forces the fit loop to one step per
    graph replay.  Step g (0-based from the first batch of epoch 0) uses
    ``lr * (1/size) * ((g + 1) / steps_per_epoch * (size - 1) / warmup_epochs + 1)``;
    ``optimizer.lr`` is kept at the value of the epoch's last step for the epoch logs and
    for later callbacks (ReduceLROnPlateau sees it, as with Horovod).  ``warmup_epochs=0``
    (the reference default) is a no-op."""
    needs_batch_logs = False

    def __init__(self, warmup_epochs=5, momentum_correction=True, steps_per_epoch=None, verbose=0):
        super().__init__()
        self.warmup_epochs = warmup_epochs
        # Horovod scales the momentum by new_lr / old_lr while the LR ramps (momentum
        # correction); that matters only for a momentum optimizer, and the device-side ramp
        # has no per-step hook for it -- refuse loudly instead of silently dropping it
        self.momentum_correction = momentum_correction
        self.steps_per_epoch = steps_per_epoch
        self.verbose = verbose
        self.initial_lr = None

    def _spe(self):
        if self.steps_per_epoch:
            return int(self.steps_per_epoch)
        if self.params.get("steps"):
            return int(self.params["steps"])
        if self.params.get("samples") and self.params.get("batch_size"):
            return -(-int(self.params["samples"]) // int(self.params["batch_size"]))
        raise ValueError("LearningRateWarmupCallback: steps per epoch unknown (pass steps_per_epoch)")

    def on_train_begin(self, logs=None):
        if self.warmup_epochs <= 0:
            return
        self.initial_lr = float(get_value(self.model.optimizer.lr))
        self._n = self._spe()
        ex = self.model._executor
        base = getattr(self.model.optimizer, "_base_optimizer", self.model.optimizer)
        # the ramp is anchored at epoch 0 (as Horovod's, which uses the absolute epoch): a
        # fit() resumed at initial_epoch > 0 continues the ramp where it stands, and one
        # resumed past the warmup window does no warmup at all
        e0 = int(self.params.get("initial_epoch", 0) or 0)
        t0 = int(base.iterations) - e0 * self._n
        window = int(round(self.warmup_epochs * self._n))
        ramping = window > 0 and e0 * self._n < window
        if (ramping and self.momentum_correction
                and float(getattr(base, "momentum", 0.0) or 0.0) > 0.0):
            # only while the LR actually ramps does momentum correction change anything
            raise NotImplementedError("LearningRateWarmupCallback(momentum_correction=True) with a momentum "
                                      "optimizer: pass momentum_correction=False")
        ex.set_lr_warmup(t0, window, self._n, dist.size(), float(self.warmup_epochs), self.initial_lr)

    def on_epoch_end(self, epoch, logs=None):
        if self.warmup_epochs <= 0 or self.initial_lr is None or epoch >= self.warmup_epochs:
            return
        from ..models.executor_base import warmup_lr
        g = min((epoch + 1) * self._n, int(round(self.warmup_epochs * self._n))) - 1
        lr = warmup_lr(g, self._n, dist.size(), float(self.warmup_epochs), self.initial_lr)
        set_value(self.model.optimizer.lr, lr)
        if logs is not None:
            logs["lr"] = lr
        if epoch == self.warmup_epochs - 1 and self.verbose > 0:
            print("\nEpoch %d: gradual learning rate warmup to %g done." % (epoch + 1, lr))

    def on_train_end(self, logs=None):
        if self.warmup_epochs > 0 and self.model is not None and self.model._executor is not None:
            self.model._executor.set_lr_warmup(0, 0, 1, 1, 1.0, 0.0)
