"""Keras-2.2-compatible callbacks.

Used by ``rpv.train_model`` (``rpv.py:80-101``: ReduceLROnPlateau, ModelCheckpoint,
user callbacks) and by the engine-side ``IPyParallelLogger`` (``mlextras.py:8-33``).
Ordering in ``fit`` follows Keras: BaseLogger -> ProgbarLogger -> user callbacks ->
History, so Horovod's MetricAverage (user list) runs before ReduceLROnPlateau and
History records the averaged values (``rpv.py:83-98``).

Attribution: ``ReduceLROnPlateau``, ``EarlyStopping``, ``ModelCheckpoint`` and ``CSVLogger``
re-implement the documented behaviour of the Keras 2.2 callbacks of the same names (Keras,
MIT License, Copyright (c) 2015-2018 the Keras authors) so that training runs reproduce the
reference's LR schedule / stopping decisions bit for bit.
"""
from __future__ import annotations

import csv
import math
import os
import sys
import time
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np

from ..optim import get_value, set_value


class Callback:
    def __init__(self):
        self.validation_data = None
        self.model = None
        self.params: Dict = {}

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_batch_begin(self, batch, logs=None): pass
    def on_batch_end(self, batch, logs=None): pass
    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass


def wants_batch_logs(cb: Callback) -> bool:
    """True if the callback consumes per-batch metric values (forces a device sync per
    batch).  Built-ins that only need epoch aggregates opt out."""
    if getattr(cb, "needs_batch_logs", None) is not None:
        return bool(cb.needs_batch_logs)
    return type(cb).on_batch_end is not Callback.on_batch_end


class CallbackList:
    def __init__(self, callbacks: Optional[List[Callback]] = None):
        self.callbacks = list(callbacks or [])

    def append(self, cb):
        self.callbacks.append(cb)

    def set_params(self, params):
        for c in self.callbacks:
            c.set_params(params)

    def set_model(self, model):
        for c in self.callbacks:
            c.set_model(model)

    def _call(self, name, *args):
        for c in self.callbacks:
            getattr(c, name)(*args)

    def on_epoch_begin(self, epoch, logs=None): self._call("on_epoch_begin", epoch, logs if logs is not None else {})
    def on_epoch_end(self, epoch, logs=None): self._call("on_epoch_end", epoch, logs if logs is not None else {})
    def on_batch_begin(self, batch, logs=None): self._call("on_batch_begin", batch, logs if logs is not None else {})
    def on_batch_end(self, batch, logs=None): self._call("on_batch_end", batch, logs if logs is not None else {})
    def on_train_begin(self, logs=None): self._call("on_train_begin", logs if logs is not None else {})
    def on_train_end(self, logs=None): self._call("on_train_end", logs if logs is not None else {})

    def __iter__(self):
        return iter(self.callbacks)

    @property
    def batch_logs_needed(self) -> bool:
        return any(wants_batch_logs(c) for c in self.callbacks)

    @property
    def batch_begin_needed(self) -> bool:
        # overridden in the class, or set on the instance (LambdaCallback(on_batch_begin=...))
        return any(type(c).on_batch_begin is not Callback.on_batch_begin or "on_batch_begin" in vars(c)
                   for c in self.callbacks)


class History(Callback):
    needs_batch_logs = False

    def on_train_begin(self, logs=None):
        self.epoch = []
        self.history = {}

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        self.epoch.append(epoch)
        for k, v in logs.items():
            self.history.setdefault(k, []).append(v)


def _fmt(v) -> str:
    return " %.4f" % v if abs(v) > 1e-3 else " %.4e" % v


class ProgbarLogger(Callback):
    """verbose=1: progress bar ``64000/64000 [====...] - 56s 880us/step - loss: ...``
    (``Train_rpv.ipynb:306``); verbose=2: one line per epoch ``" - 11s - loss: ..."``
    (``DistTrain_mnist.ipynb:343``)."""
    needs_batch_logs = False

    def __init__(self, stream=None):
        super().__init__()
        self.stream = stream

    def _out(self):
        return self.stream or sys.stdout

    def on_train_begin(self, logs=None):
        self.verbose = self.params.get("verbose", 1)
        self.epochs = self.params.get("epochs", 1)

    def on_epoch_begin(self, epoch, logs=None):
        if self.verbose:
            print("Epoch %d/%d" % (epoch + 1, self.epochs), file=self._out())
        self._start = time.time()
        self._last_update = 0.0
        self.target = self.params.get("samples") or 0

    def progress(self, seen, values):
        """Mid-epoch update from the fit loop (throttled)."""
        if self.verbose != 1:
            return
        now = time.time()
        if now - self._last_update < 0.5 and seen < self.target:
            return
        self._last_update = now
        self._draw(seen, values, final=False)

    def _draw(self, seen, values, final):
        width = 30
        numdigits = int(np.floor(np.log10(max(self.target, 1)))) + 1
        bar = ("%" + str(numdigits) + "d/%d [") % (seen, self.target)
        prog = float(seen) / max(self.target, 1)
        w = int(width * prog)
        if w > 0:
            bar += "=" * (w - 1)
            bar += "=" if seen >= self.target else ">"
        bar += "." * (width - w) + "]"
        elapsed = time.time() - self._start
        if final:
            per = elapsed / max(seen, 1)
            if per >= 1:
                info = " - %.0fs %.0fs/step" % (elapsed, per)
            elif per >= 1e-3:
                info = " - %.0fs %.0fms/step" % (elapsed, per * 1e3)
            else:
                info = " - %.0fs %.0fus/step" % (elapsed, per * 1e6)
        else:
            eta = elapsed / max(seen, 1) * (self.target - seen)
            info = " - ETA: %ds" % eta
        for k, v in values:
            info += " - %s:" % k + _fmt(v)
        end = "\n" if final else "\r"
        self._out().write("\r" + bar + info + end if not final else "\r" + bar + info + "\n")
        self._out().flush()

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        vals = [(k, logs[k]) for k in self.params.get("metrics", []) if k in logs]
        if self.verbose == 1:
            self._draw(self.target, vals, final=True)
        elif self.verbose == 2:
            info = " - %.0fs" % (time.time() - self._start)
            for k, v in vals:
                info += " - %s:" % k + _fmt(v)
            print(info, file=self._out())
            self._out().flush()


class ModelCheckpoint(Callback):
    """Whole-model Keras-HDF5 save every epoch (``rpv.py:100-101``)."""
    needs_batch_logs = False

    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False,
                 save_weights_only=False, mode="auto", period=1):
        super().__init__()
        self.filepath = filepath
        self.monitor = monitor
        self.verbose = verbose
        self.save_best_only = save_best_only
        self.save_weights_only = save_weights_only
        self.period = period
        self.epochs_since_last_save = 0
        if mode not in ("auto", "min", "max"):
            mode = "auto"
        if mode == "min" or (mode == "auto" and not ("acc" in monitor or monitor.startswith("fmeasure"))):
            self.monitor_op, self.best = np.less, np.inf
        else:
            self.monitor_op, self.best = np.greater, -np.inf

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        self.epochs_since_last_save += 1
        if self.epochs_since_last_save < self.period:
            return
        self.epochs_since_last_save = 0
        filepath = self.filepath.format(epoch=epoch + 1, **logs)
        if self.save_best_only:
            current = logs.get(self.monitor)
            if current is None or not self.monitor_op(current, self.best):
                if self.verbose > 0 and current is not None:
                    print("\nEpoch %05d: %s did not improve from %0.5f" % (epoch + 1, self.monitor, self.best))
                return
            if self.verbose > 0:
                print("\nEpoch %05d: %s improved from %0.5f to %0.5f, saving model to %s"
                      % (epoch + 1, self.monitor, self.best, current, filepath))
            self.best = current
        elif self.verbose > 0:
            print("\nEpoch %05d: saving model to %s" % (epoch + 1, filepath))
        if self.save_weights_only:
            self.model.save_weights(filepath, overwrite=True)
        else:
            self.model.save(filepath, overwrite=True)


class ReduceLROnPlateau(Callback):
    """Keras defaults: monitor val_loss, factor 0.1, min_delta 1e-4, cooldown 0, min_lr 0;
    writes ``lr`` into the epoch logs (``rpv.py:94-98``).

    Attribution: the decision logic follows Keras 2.2's ``ReduceLROnPlateau``
    (keras/callbacks.py, MIT license, (c) François Chollet and contributors) step for step,
    so that the reference's LR trajectories are reproduced exactly."""
    needs_batch_logs = False

    def __init__(self, monitor="val_loss", factor=0.1, patience=10, verbose=0, mode="auto",
                 min_delta=1e-4, cooldown=0, min_lr=0, **kwargs):
        super().__init__()
        if "epsilon" in kwargs:
            min_delta = kwargs.pop("epsilon")
        if factor >= 1.0:
            raise ValueError("ReduceLROnPlateau does not support a factor >= 1.0.")
        self.monitor, self.factor, self.min_lr = monitor, factor, min_lr
        self.min_delta, self.patience, self.verbose = min_delta, patience, verbose
        self.cooldown, self.mode = cooldown, mode
        self._reset()

    def _reset(self):
        if self.mode == "min" or (self.mode == "auto" and "acc" not in self.monitor):
            self.monitor_op = lambda a, b: np.less(a, b - self.min_delta)
            self.best = np.inf
        else:
            self.monitor_op = lambda a, b: np.greater(a, b + self.min_delta)
            self.best = -np.inf
        self.cooldown_counter = 0
        self.wait = 0

    def on_train_begin(self, logs=None):
        self._reset()

    def on_epoch_end(self, epoch, logs=None):
        logs = logs if logs is not None else {}
        logs["lr"] = get_value(self.model.optimizer.lr)
        current = logs.get(self.monitor)
        if current is None:
            return
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.wait = 0
        if self.monitor_op(current, self.best):
            self.best = current
            self.wait = 0
        elif not self.cooldown_counter > 0:
            self.wait += 1
            if self.wait >= self.patience:
                old_lr = float(get_value(self.model.optimizer.lr))
                if old_lr > self.min_lr:
                    new_lr = max(old_lr * self.factor, self.min_lr)
                    set_value(self.model.optimizer.lr, new_lr)
                    if self.verbose > 0:
                        print("\nEpoch %05d: ReduceLROnPlateau reducing learning rate to %s." % (epoch + 1, new_lr))
                    self.cooldown_counter = self.cooldown
                    self.wait = 0


class EarlyStopping(Callback):
    """Keras 2.2 ``EarlyStopping`` semantics (keras/callbacks.py, MIT license, (c) François
    Chollet and contributors; logic followed step for step for bit-identical stopping)."""
    needs_batch_logs = False

    def __init__(self, monitor="val_loss", min_delta=0, patience=0, verbose=0, mode="auto",
                 baseline=None, restore_best_weights=False):
        super().__init__()
        self.monitor, self.patience, self.verbose = monitor, patience, verbose
        self.baseline, self.min_delta = baseline, abs(min_delta)
        self.restore_best_weights = restore_best_weights
        if mode == "min" or (mode == "auto" and "acc" not in monitor):
            self.monitor_op = np.less
            self.min_delta *= -1
        else:
            self.monitor_op = np.greater

    def on_train_begin(self, logs=None):
        self.wait = 0
        self.stopped_epoch = 0
        self.best = self.baseline if self.baseline is not None else (
            np.inf if self.monitor_op == np.less else -np.inf)
        self.best_weights = None

    def on_epoch_end(self, epoch, logs=None):
        current = (logs or {}).get(self.monitor)
        if current is None:
            return
        if self.monitor_op(current - self.min_delta, self.best):
            self.best = current
            self.wait = 0
            if self.restore_best_weights:
                self.best_weights = self.model.get_weights()
        else:
            self.wait += 1
            if self.wait >= self.patience:
                self.stopped_epoch = epoch
                self.model.stop_training = True
                if self.restore_best_weights and self.best_weights is not None:
                    self.model.set_weights(self.best_weights)

    def on_train_end(self, logs=None):
        if self.stopped_epoch > 0 and self.verbose > 0:
            print("Epoch %05d: early stopping" % (self.stopped_epoch + 1))


class LearningRateScheduler(Callback):
    needs_batch_logs = False

    def __init__(self, schedule, verbose=0):
        super().__init__()
        self.schedule, self.verbose = schedule, verbose

    def on_epoch_begin(self, epoch, logs=None):
        lr = float(get_value(self.model.optimizer.lr))
        try:
            lr = self.schedule(epoch, lr)
        except TypeError:
            lr = self.schedule(epoch)
        set_value(self.model.optimizer.lr, lr)
        if self.verbose > 0:
            print("\nEpoch %05d: LearningRateScheduler setting learning rate to %s." % (epoch + 1, lr))


class TerminateOnNaN(Callback):
    """Epoch-granular NaN guard (checking per batch would force a device sync)."""
    needs_batch_logs = False

    def on_epoch_end(self, epoch, logs=None):
        loss = (logs or {}).get("loss")
        if loss is not None and (np.isnan(loss) or np.isinf(loss)):
            print("Epoch %d: Invalid loss, terminating training" % epoch)
            self.model.stop_training = True


class CSVLogger(Callback):
    needs_batch_logs = False

    def __init__(self, filename, separator=",", append=False):
        super().__init__()
        self.filename, self.sep, self.append = filename, separator, append
        self.keys = None

    def on_train_begin(self, logs=None):
        mode = "a" if self.append and os.path.exists(self.filename) else "w"
        self.fh = open(self.filename, mode, newline="")
        self.writer = None

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        if self.keys is None:
            self.keys = sorted(logs.keys())
        if self.writer is None:
            self.writer = csv.DictWriter(self.fh, fieldnames=["epoch"] + self.keys, delimiter=self.sep)
            if not self.append:
                self.writer.writeheader()
        row = OrderedDict({"epoch": epoch})
        row.update((k, logs.get(k, "NA")) for k in self.keys)
        self.writer.writerow(row)
        self.fh.flush()

    def on_train_end(self, logs=None):
        self.fh.close()


class LambdaCallback(Callback):
    def __init__(self, on_epoch_begin=None, on_epoch_end=None, on_batch_begin=None, on_batch_end=None,
                 on_train_begin=None, on_train_end=None, **kw):
        super().__init__()
        nop = lambda *a, **k: None
        self.on_epoch_begin = on_epoch_begin or nop
        self.on_epoch_end = on_epoch_end or nop
        self.on_train_begin = on_train_begin or nop
        self.on_train_end = on_train_end or nop
        if on_batch_begin is not None:
            self.on_batch_begin = on_batch_begin
        if on_batch_end is not None:
            self.on_batch_end = on_batch_end
        self.needs_batch_logs = on_batch_end is not None
