"""Tracing / profiling hooks (SURVEY.md §5 "Tracing / profiling").

The reference had only Keras' per-epoch seconds and ``%%time`` cells.  Here:

* ``StepTimer``       -- HIP-event timing of device work (no host sync per step: events are
                         recorded on the stream and read once at ``summary()``).
* ``ThroughputLogger``-- a Keras callback adding ``img_per_sec`` (per GPU) and
                         ``img_per_sec_node`` (all ranks) to the epoch logs, so throughput
                         shows up in History and the farm's ``publish_data`` stream (epoch
                         wall time, validation pass included, as Keras' epoch seconds).
* ``trace(path)``     -- a ``torch.profiler`` context writing a Chrome trace of host + HIP
                         activity (kernel launches, RCCL calls) for one region.

For per-kernel device timings use ``rocprofv3 --kernel-trace --stats`` (``scripts/
prof_model.sh``); those summaries are what ``profiles/`` holds.
"""
from __future__ import annotations

import contextlib
import time
from typing import Dict, List, Optional

import torch

from ..train.callbacks import Callback


class StepTimer:
    """Accumulates device time of ``with timer.region("name"):`` blocks via HIP events."""

    def __init__(self, device=None):
        self.enabled = torch.cuda.is_available()
        self._events: Dict[str, List] = {}
        self._host: Dict[str, List[float]] = {}

    @contextlib.contextmanager
    def region(self, name: str):
        if self.enabled:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            yield
            e.record()
            self._events.setdefault(name, []).append((s, e))
        else:
            t0 = time.perf_counter()
            yield
            self._host.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)

    def summary(self) -> Dict[str, Dict[str, float]]:
        """{name: {calls, total_ms, mean_ms}} (synchronises once)."""
        out = {}
        if self._events:
            torch.cuda.synchronize()
        for name, evs in self._events.items():
            ms = [s.elapsed_time(e) for s, e in evs]
            out[name] = {"calls": len(ms), "total_ms": sum(ms), "mean_ms": sum(ms) / len(ms)}
        for name, ms in self._host.items():
            out[name] = {"calls": len(ms), "total_ms": sum(ms), "mean_ms": sum(ms) / len(ms)}
        return out

    def reset(self):
        self._events.clear()
        self._host.clear()


class ThroughputLogger(Callback):
    """Adds ``epoch_sec``, ``img_per_sec`` and ``img_per_sec_node`` to each epoch's logs
    (training images over the epoch's wall time)."""

    needs_batch_logs = False

    def __init__(self):
        super().__init__()
        self._t0 = None
        self.history: List[Dict[str, float]] = []

    def on_epoch_begin(self, epoch, logs=None):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._t0 = time.perf_counter()

    def on_epoch_end(self, epoch, logs=None):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dt = time.perf_counter() - self._t0
        n = (self.params or {}).get("samples") or 0
        from ..parallel import state
        st = state.current()
        size = st.size if st is not None else 1
        rec = {"epoch_sec": dt, "img_per_sec": n / dt if dt > 0 else 0.0}
        rec["img_per_sec_node"] = rec["img_per_sec"] * size
        self.history.append(rec)
        if logs is not None:
            logs.update(rec)


@contextlib.contextmanager
def trace(path: str, with_stack: bool = False):
    """``with trace("step.json"): model.fit(...)`` -> Chrome trace of the region."""
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    with profile(activities=acts, with_stack=with_stack) as prof:
        yield prof
    prof.export_chrome_trace(path)
