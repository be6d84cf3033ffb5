"""Random hyper-parameter search over the task farm.

The samplers reproduce the notebooks' ``np.random`` call order exactly, so with the
same seed they yield the same trial lists (golden facts):

* ``mnist_trials``  -- ``DistHPO_mnist.ipynb:137-150`` / ``HPO_mnist.ipynb:112-127`` /
  ``DistWidgetHPO_mnist.ipynb:143-156``: h1, h2 ∈ {4..64}, h3 ∈ {8..128},
  dropout ~ U(0,1), optimizer ∈ {Adadelta, Adam, Nadam}
* ``rpv_trials``    -- ``DistHPO_rpv.ipynb:91-106`` / ``DistWidgetHPO_rpv.ipynb:110-125``:
  conv (h1, h2, h3), fc ∈ {32..256}, lr ∈ {1e-4, 1e-3, 1e-2}, dropout, optimizer

``submit_trials`` sends one ``build_and_train(**trial)`` per trial to a
load-balanced view (``DistHPO_mnist.ipynb:240-255``): eight MI355X engines run eight
trials at a time.  ``collect`` / ``best_trial`` / ``runtime_seconds`` are the analysis
steps of the notebooks (``:272``, ``:344``, ``:360-361``, ``DistHPO_rpv.ipynb:217``).
"""
from __future__ import annotations

import time
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np

MNIST_H12 = [4, 8, 16, 32, 64]
MNIST_H3 = [8, 16, 32, 64, 128]
OPTIMIZERS = ["Adadelta", "Adam", "Nadam"]
RPV_FC = [32, 64, 128, 256]
RPV_LR = [0.0001, 0.001, 0.01]


def mnist_trials(n_trials: int, seed: Optional[int] = 0) -> List[Dict[str, Any]]:
    if seed is not None:
        np.random.seed(seed)
    h1 = np.random.choice(MNIST_H12, size=n_trials)
    h2 = np.random.choice(MNIST_H12, size=n_trials)
    h3 = np.random.choice(MNIST_H3, size=n_trials)
    dropout = np.random.rand(n_trials)
    opt = np.random.choice(OPTIMIZERS, size=n_trials)
    return [dict(h1=int(h1[i]), h2=int(h2[i]), h3=int(h3[i]), dropout=float(dropout[i]), optimizer=str(opt[i]))
            for i in range(n_trials)]


def rpv_trials(n_trials: int, seed: Optional[int] = 0) -> List[Dict[str, Any]]:
    if seed is not None:
        np.random.seed(seed)
    h1 = np.random.choice(MNIST_H12, size=n_trials)
    h2 = np.random.choice(MNIST_H12, size=n_trials)
    h3 = np.random.choice(MNIST_H3, size=n_trials)
    conv = np.stack([h1, h2, h3], axis=1)
    fc = np.random.choice(RPV_FC, size=(n_trials, 1))
    lr = np.random.choice(RPV_LR, size=n_trials)
    dropout = np.random.rand(n_trials)
    opt = np.random.choice(OPTIMIZERS, size=n_trials)
    return [dict(conv_sizes=[int(v) for v in conv[i]], fc_sizes=[int(v) for v in fc[i]], lr=float(lr[i]),
                 dropout=float(dropout[i]), optimizer=str(opt[i])) for i in range(n_trials)]


def describe(trial: Dict[str, Any]) -> str:
    """One-line trial label as the notebooks print them (``64-8-128 dropout 0.020 Nadam``)."""
    if "conv_sizes" in trial:
        sizes = "-".join(str(v) for v in list(trial["conv_sizes"]) + list(trial["fc_sizes"]))
        return "%s lr %g dropout %.3f %s" % (sizes, trial["lr"], trial["dropout"], trial["optimizer"])
    return "%d-%d-%d dropout %.3f %s" % (trial["h1"], trial["h2"], trial["h3"], trial["dropout"], trial["optimizer"])


def submit_trials(view, fn: Callable, trials: Sequence[Dict[str, Any]], with_index: bool = False,
                  **common) -> List:
    """``[view.apply(fn, **trial, **common)]``; with ``with_index`` the trial index is passed
    as ``trial_index`` (checkpoint file naming, ``DistHPO_mnist.ipynb:248``)."""
    out = []
    for i, t in enumerate(trials):
        kw = dict(common)
        kw.update(t)
        if with_index:
            kw["trial_index"] = i
        out.append(view.apply(fn, **kw))
    return out


def wait_progress(results: Sequence, interval: float = 5.0, timeout: Optional[float] = None,
                  printer: Callable[[str], None] = print) -> None:
    """Poll until every trial finishes, printing ``done/total`` (``DistHPO_mnist.ipynb:272``)."""
    t0 = time.time()
    last = -1
    while True:
        done = sum(1 for r in results if r.ready())
        if done != last:
            printer("%d / %d trials done" % (done, len(results)))
            last = done
        if done == len(results):
            return
        if timeout is not None and time.time() - t0 > timeout:
            raise TimeoutError("%d trials still running" % (len(results) - done))
        time.sleep(interval)


def collect(results: Sequence) -> List[Optional[Dict[str, List[float]]]]:
    """History dicts of finished trials (None for failed ones, instead of raising)."""
    out = []
    for r in results:
        try:
            out.append(r.get())
        except Exception:
            out.append(None)
    return out


def best_trial(histories: Sequence[Optional[Dict[str, List[float]]]], key: str = "val_acc",
               mode: str = "max", reduce: str = "last"):
    """Index and score of the best trial by ``key`` (the ``[-1]`` epoch value by default,
    ``DistHPO_mnist.ipynb:360-361``); failed trials are skipped."""
    best_i, best = None, None
    for i, h in enumerate(histories):
        if not h or key not in h or not h[key]:
            continue
        v = h[key][-1] if reduce == "last" else (max(h[key]) if mode == "max" else min(h[key]))
        if best is None or (v > best if mode == "max" else v < best):
            best_i, best = i, v
    return best_i, best


def runtime_seconds(results: Sequence) -> np.ndarray:
    """Per-trial wall time ``completed - started`` (``DistHPO_rpv.ipynb:217``)."""
    return np.asarray([(r.completed - r.started).total_seconds() if r.completed and r.started else np.nan
                       for r in results])
