"""Engine-side helpers (``mlextras.py:1-43``).

``IPyParallelLogger`` streams a trial's training progress to the notebook through the
farm's ``publish_data`` (SURVEY.md Appendix B.4 schema): ``{"status": "Begin Training" |
"Begin Epoch" | "Ended Epoch" | "Ended Training", "epoch": int, "history": {acc, loss,
val_acc, val_loss, epoch}}``; the client sees the merged dict as ``AsyncResult.data``
(``hpo_widgets.py:260``).  Outside a farm task publishing is a no-op.

``configure_session`` replaced a TF CPU session with inter/intra-op thread counts
(``mlextras.py:35-43``).  On MI355X the kernels run on the GPU; what remains is the host
thread budget for the framework's CPU side (data prep, the CPU reference backend), taken
from the same ``NUM_INTER_THREADS`` / ``NUM_INTRA_THREADS`` variables.
"""
from __future__ import annotations

import os
from typing import Dict

from ..farm.engine import publish_data
from ..train.callbacks import Callback


class IPyParallelLogger(Callback):
    needs_batch_logs = False

    def __init__(self):
        super().__init__()
        self.history: Dict[str, list] = {}

    def _pub(self, status, epoch=None):
        msg = {"status": status, "history": {k: list(v) for k, v in self.history.items()}}
        if epoch is not None:
            msg["epoch"] = epoch
        publish_data(msg)

    def on_train_begin(self, logs=None):
        self.history = {"acc": [], "loss": [], "val_acc": [], "val_loss": [], "epoch": []}
        self._pub("Begin Training")

    def on_train_end(self, logs=None):
        self._pub("Ended Training")

    def on_epoch_begin(self, epoch, logs=None):
        self._pub("Begin Epoch", epoch)

    def on_epoch_end(self, epoch, logs=None):
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(float(v))
        self.history["epoch"].append(epoch)
        self._pub("Ended Epoch", epoch)


class SessionConfig:
    def __init__(self, inter_op_parallelism_threads: int, intra_op_parallelism_threads: int):
        self.inter_op_parallelism_threads = inter_op_parallelism_threads
        self.intra_op_parallelism_threads = intra_op_parallelism_threads

    def __repr__(self):
        return "SessionConfig(inter=%d, intra=%d)" % (self.inter_op_parallelism_threads,
                                                      self.intra_op_parallelism_threads)


def configure_session() -> SessionConfig:
    import torch
    inter = int(os.environ.get("NUM_INTER_THREADS", 2))
    intra = int(os.environ.get("NUM_INTRA_THREADS", 32))
    intra = max(1, min(intra, os.cpu_count() or intra))
    torch.set_num_threads(intra)
    try:
        torch.set_num_interop_threads(inter)
    except RuntimeError:      # can only be set once per process, before any parallel work
        pass
    return SessionConfig(inter, intra)
