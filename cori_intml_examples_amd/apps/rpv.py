"""RPV recipe: data loading, model factory and training driver (the reference's
``rpv.py:1-106``, used by every RPV notebook and by ``train_rpv``).

Differences from the reference, all deliberate:
* ``train_model`` copies ``callbacks`` instead of appending to a shared mutable default
  (the reference's ``callbacks=[]`` default grows across calls, ``rpv.py:79,83,94,101``).
* Rank-0-only checkpoint writes under data parallelism (the reference writes from every
  rank; the fix is recommended but commented out at ``DistTrain_mnist.ipynb:497-499``).
* ``load_dataset`` falls back to a synthetic dataset of the same schema when the input
  directory does not exist and ``synthetic=True`` (there is no Cori scratch here).
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np

from ..io import datasets as _ds
from ..train import callbacks as _cb
from .zoo import rpv_cnn

N_TRAIN, N_VALID, N_TEST = 412416, 137471, 137471     # rpv.py:27


def load_file(filename: str, n_samples: int):
    """``all_events/{hist,y,weight}`` of one HDF5 file, first ``n_samples`` events, with a
    channel axis added (``rpv.py:19-25``)."""
    return _ds.load_file(filename, n_samples)


def load_dataset(path: str, n_train: int = N_TRAIN, n_valid: int = N_VALID, n_test: int = N_TEST,
                 synthetic: bool = False, channels: int = 1, seed: int = 0):
    """``(train, valid, test)`` tuples of ``(hist, y, weight)`` (``rpv.py:27-36``)."""
    if synthetic and not os.path.exists(os.path.join(path, "train.h5")):
        out = []
        for i, n in enumerate((n_train, n_valid, n_test)):
            out.append(_ds.synthetic_rpv(n, channels=channels, seed=seed + i))
        return tuple(out)
    return _ds.load_dataset(path, n_train, n_valid, n_test)


def build_model(input_shape, conv_sizes=(8, 16, 32), fc_sizes=(64,), dropout=0.5, optimizer="Adam",
                lr=0.001, use_horovod=False, device=None):
    """Functional CNN ``'RPVClassifier'`` (``rpv.py:38-71``): ``[Conv3x3 same+ReLU,
    MaxPool2]`` per conv size, Dropout, Flatten, ``[Dense+ReLU, Dropout]`` per fc size,
    Dense(1, sigmoid); BCE + accuracy; optimizer by name with ``lr``, Horovod-wrapped
    when ``use_horovod``."""
    return rpv_cnn(tuple(input_shape), conv_sizes=list(conv_sizes), fc_sizes=list(fc_sizes), dropout=dropout,
                   optimizer=optimizer, lr=lr, use_horovod=use_horovod, device=device)


def train_model(model, train_input, train_labels, valid_input, valid_labels, batch_size, n_epochs,
                lr_warmup_epochs=0, lr_reduce_patience=8, checkpoint_file=None, use_horovod=False,
                verbose=2, callbacks: Optional[List] = None):
    """``rpv.py:74-106``: Horovod Broadcast(0) / MetricAverage / LR warmup first (so
    ReduceLROnPlateau sees rank-averaged ``val_loss``), then ReduceLROnPlateau(patience),
    then an optional whole-model checkpoint each epoch."""
    cbs = list(callbacks or [])
    if use_horovod:
        from ..parallel import hvd
        cbs += [hvd.callbacks.BroadcastGlobalVariablesCallback(0),
                hvd.callbacks.MetricAverageCallback(),
                hvd.callbacks.LearningRateWarmupCallback(warmup_epochs=lr_warmup_epochs, verbose=1)]
    cbs.append(_cb.ReduceLROnPlateau(patience=lr_reduce_patience, verbose=1))
    if checkpoint_file is not None:
        rank0 = True
        if use_horovod:
            from ..parallel import hvd
            rank0 = hvd.rank() == 0
        if rank0:
            cbs.append(_cb.ModelCheckpoint(checkpoint_file))
    return model.fit(x=train_input, y=train_labels, batch_size=batch_size, epochs=n_epochs,
                     validation_data=(valid_input, valid_labels), callbacks=cbs, verbose=verbose)


def classification_report(labels, outputs, weights=None, threshold=0.5):
    """Accuracy / purity (precision) / efficiency (recall) as printed by the RPV analysis
    cells (``DistTrain_rpv.ipynb:378-396,435-437``), optionally event-weighted."""
    labels = np.asarray(labels).reshape(-1)
    pred = (np.asarray(outputs).reshape(-1) > threshold).astype(np.float32)
    w = np.ones_like(labels, dtype=np.float64) if weights is None else np.asarray(weights, np.float64).reshape(-1)
    tp = float((w * (pred == 1) * (labels == 1)).sum())
    fp = float((w * (pred == 1) * (labels == 0)).sum())
    fn = float((w * (pred == 0) * (labels == 1)).sum())
    acc = float((w * (pred == labels)).sum() / w.sum())
    return {"accuracy": acc, "purity": tp / max(tp + fp, 1e-30), "efficiency": tp / max(tp + fn, 1e-30)}
