"""Headless data model of the live HPO dashboard (``hpo_widgets.py``, SURVEY.md §2.1
C9a-e, §3.4).  Everything the widgets show lives here, so it is testable without a
browser; ``widgets/ui.py`` only renders it (ipywidgets/bqplot/qgrid when installed).

* ``ModelPlotTable``  column-major table; ``append_row`` fills missing columns with None
                      (``hpo_widgets.py:441-484``).
* ``ModelTaskData``   per-trial store: plot table + status dict (``:410-438``).
* ``ModelController`` trial scheduler facade over the farm's load-balanced view
                      (``:373-407``) -- with WORKING ``stop_model`` / ``restart_model``
                      (the reference's were stubs): stop = ``AsyncResult.abort`` (cooperative
                      flag, then engine hard-kill after the grace period); restart = stop +
                      resubmit with the same parameters.
* ``PlotModel``       the state of one ``ModelPlot``: one (x, y) series per metric and
                      the axis extents grown to the data (``:115-142``).
* ``ParamSpanModel``  the parameter table (pandas), one ModelTaskData + PlotModel per
                      row, and ``poll()``: one pass of the reference's 1 Hz update loop
                      (``:254-323``) applying ``AsyncResult.data`` (the ``publish_data``
                      stream of ``IPyParallelLogger``) to the table and plots.

Concurrency fixes vs the reference (SURVEY.md §5 "Race detection"): all state mutation
happens under one lock; the polling thread starts on ``submit_computations`` (not in the
constructor) and stops cleanly (``stop_polling``); new history rows are appended exactly
once (the reference re-appended the last row on every update).
"""
from __future__ import annotations

import copy
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np


class ModelPlotTable:
    """Per-epoch metric records of one trial.

    Storage is row-major: one tuple per appended record, in the order of ``columns``;
    a column added later is back-filled with ``None``.  ``rows`` / ``to_dict`` present
    the column-major view the plot consumes (one list per column)."""

    def __init__(self, column_names: Sequence[str]):
        self._order: List[str] = []
        self._slot: Dict[str, int] = {}
        self._records: List[tuple] = []
        for name in column_names:
            self._add_name(name)

    def _add_name(self, name: str) -> None:
        if name in self._slot:
            raise KeyError("duplicate column name %r" % (name,))
        self._slot[name] = len(self._order)
        self._order.append(name)

    @property
    def columns(self) -> List[str]:
        return list(self._order)

    @property
    def num_rows(self) -> int:
        return len(self._records)

    def column(self, name: str) -> list:
        j = self._slot[name]
        return [rec[j] if j < len(rec) else None for rec in self._records]

    @property
    def rows(self) -> List[list]:
        """Column-major view: ``rows[j]`` holds every value of ``columns[j]``."""
        return [self.column(n) for n in self._order]

    def append_column(self, name: str, vals: Optional[Sequence] = None) -> None:
        """New column, back-filled from ``vals`` (one per existing record) or with None."""
        fill = list(vals) if vals is not None and len(vals) else None
        if fill is not None and len(fill) != len(self._records):
            raise ValueError("column %r has %d values, table has %d rows" % (name, len(fill), len(self._records)))
        self._add_name(name)
        if fill is not None:
            # records older than an earlier value-less column are short: pad them to the new
            # column's slot so the value lands under its own name
            j = self._slot[name]
            self._records = [rec + (None,) * (j - len(rec)) + (v,) for rec, v in zip(self._records, fill)]
        # (without values, older records are shorter than ``columns``: read as None)

    def append_row(self, row: Dict[str, Any]) -> None:
        """One record; keys that are not columns are ignored, missing columns are None."""
        self._records.append(tuple(row.get(n) for n in self._order))

    def to_dict(self) -> Dict[str, list]:
        return {n: self.column(n) for n in self._order}


class ModelTaskData:
    """Everything the dashboard knows about one trial: its metric records and its latest
    status fields, plus a revision count so a renderer can ask what changed since it
    last looked (``has_updates`` / ``clear_updates``)."""

    def __init__(self, plot_columns: Sequence[str], status_columns: Sequence[str]):
        self._metric_names = list(plot_columns)
        self._status_names = list(status_columns)
        self._table = ModelPlotTable(self._metric_names)
        self._fields: Dict[str, Any] = dict.fromkeys(self._status_names)
        self._rev, self._seen = 1, 0

    def _touch(self) -> None:
        self._rev += 1

    @property
    def has_updates(self) -> bool:
        return self._rev != self._seen

    def clear_updates(self) -> None:
        self._seen = self._rev

    @property
    def num_data_rows(self) -> int:
        return self._table.num_rows

    def get_plot_data(self) -> Dict[str, list]:
        return self._table.to_dict()

    def append_plot_data_row(self, d: Dict[str, Any]) -> None:
        self._table.append_row(d)
        self._touch()

    def set_status_data(self, d: Dict[str, Any]) -> None:
        self._fields.update(d)
        self._touch()

    def get_status_data(self) -> Dict[str, Any]:
        return dict(self._fields)

    def reset(self) -> None:
        """Forget the records and status (a restarted trial starts a fresh curve)."""
        self._table = ModelPlotTable(self._metric_names)
        self._fields = dict.fromkeys(self._status_names)
        self._touch()


class ModelController:
    """Submits one trial per model id to the farm and tracks its future."""

    def __init__(self, ipp_cluster_id: Optional[str] = None, client=None, view=None):
        if view is None:
            if client is None:
                from ..farm import Client
                client = Client(cluster_id=ipp_cluster_id)
            view = client.load_balanced_view()
        self._client = client
        self._lview = view
        self._futures: Dict[int, Any] = {}
        self._params: Dict[int, Dict[str, Any]] = {}
        self._funcs: Dict[int, Callable] = {}
        self._completed: Dict[int, Any] = {}
        self._stopped: Dict[int, Any] = {}

    def start_model(self, model_id: int, compute_func: Callable, params: Dict[str, Any]):
        self._funcs[model_id], self._params[model_id] = compute_func, dict(params)
        self._completed.pop(model_id, None)
        self._stopped.pop(model_id, None)
        self._futures[model_id] = self._lview.apply(compute_func, **params)
        return self._futures[model_id]

    def stop_model(self, model_id: int, grace: Optional[float] = None) -> None:
        fut = self._futures.pop(model_id, None)
        if fut is not None:
            if not fut.ready():
                fut.abort(grace=grace)
            self._stopped[model_id] = fut

    def restart_model(self, model_id: int, compute_func: Optional[Callable] = None,
                      params: Optional[Dict[str, Any]] = None):
        self.stop_model(model_id)
        fn = compute_func or self._funcs[model_id]
        return self.start_model(model_id, fn, params if params is not None else self._params[model_id])

    def set_model_completed(self, model_id: int) -> None:
        fut = self._futures.get(model_id)
        if fut is not None:
            self._completed[model_id] = fut

    def get_completed_models(self) -> Dict[int, Any]:
        return dict(self._completed)

    def get_running_models(self) -> Dict[int, Any]:
        """Futures still of interest: not finished, or finished but not yet marked
        completed (so their final published data is still applied once)."""
        out = {}
        for mid, fut in list(self._futures.items()):
            if mid in self._completed and fut.ready():
                del self._futures[mid]
                continue
            out[mid] = fut
        return out

    def future(self, model_id: int):
        return self._futures.get(model_id) or self._completed.get(model_id) or self._stopped.get(model_id)

    def get_resource_usage(self) -> Dict[Any, Any]:
        """Per-engine queue / running task / GPU / restarts (the reference's stub,
        ``hpo_widgets.py:366-367``)."""
        if self._client is None:
            return {}
        return self._client.queue_status()


class PlotModel:
    """Series and extents of one training-curve plot (``ModelPlot``)."""

    def __init__(self, y, x: Optional[str] = None, xlim=None, ylim=None, xlabel=None, ylabel=None, title=None):
        self.y = list(y) if isinstance(y, (list, tuple)) else [y]
        self.x = x
        self.xlim = list(xlim or [0, 1])
        self.ylim = list(ylim or [0, 1])
        self.xlabel = xlabel or "x"
        self.ylabel = ylabel or "y"
        self.title = title or "{} vs {}".format(self.ylabel, self.xlabel)
        self.series: Dict[str, Dict[str, np.ndarray]] = {k: {"x": np.zeros(0), "y": np.zeros(0)} for k in self.y}
        self.errors: List[str] = []

    def update(self, data: Dict[str, Sequence]) -> None:
        try:
            for k in self.y:
                yv = np.asarray([np.nan if v is None else v for v in data.get(k, [])], dtype=np.float64)
                if self.x and self.x in data:
                    xv = np.asarray(data[self.x], dtype=np.float64)[:len(yv)]
                else:
                    xv = np.arange(len(yv), dtype=np.float64)
                self.series[k] = {"x": xv, "y": yv}
            self._resize()
        except Exception as e:     # keep the UI alive on malformed data; record why
            self.errors.append("update failed: %r (data keys %s)" % (e, sorted(data)))

    def _resize(self) -> None:
        for s in self.series.values():
            xs, ys = s["x"], s["y"][np.isfinite(s["y"])] if len(s["y"]) else s["y"]
            if len(xs):
                self.xlim = [min(self.xlim[0], float(xs.min())), max(self.xlim[1], float(xs.max()))]
            if len(ys):
                self.ylim = [min(self.ylim[0], float(ys.min())), max(self.ylim[1], float(ys.max()))]

    @property
    def num_points(self) -> int:
        return max((len(s["y"]) for s in self.series.values()), default=0)


class ParamSpanModel:
    """Parameter-span table + per-trial data/plots + the polling logic of the dashboard."""

    METRICS = ["loss", "val_loss", "acc", "val_acc"]

    def __init__(self, compute_func: Callable, params: Dict[str, Sequence], vis_func: Optional[Callable] = None,
                 controller: Optional[ModelController] = None, ipp_cluster_id: Optional[str] = None,
                 columns: Optional[Sequence[str]] = None):
        import pandas as pd
        self.compute_func = compute_func
        self.compute_params = {k: (v.tolist() if isinstance(v, np.ndarray) else list(v)) for k, v in params.items()}
        lens = {len(v) for v in self.compute_params.values()}
        if len(lens) != 1:
            raise ValueError("all parameter lists must have the same length")
        self.n_models = lens.pop()
        self.columns = list(columns) if columns else (["status", "epoch"] + list(params) + self.METRICS)
        disp = {}
        for k, vals in self.compute_params.items():
            disp[k] = [str(v) if isinstance(v, (list, tuple)) else v for v in vals]
        df = pd.DataFrame({c: disp.get(c, [None] * self.n_models) for c in self.columns})
        df["status"] = ["Not Started"] * self.n_models
        df["epoch"] = [-1] * self.n_models
        self.table = df
        vis_func = vis_func or (lambda title: PlotModel(["loss", "val_loss", "acc", "val_acc"], x="epoch",
                                                        title=title))
        self.plots = [vis_func(title="Model {}: {}".format(i, self.params_of(i))) for i in range(self.n_models)]
        self.data = [ModelTaskData(["epoch"] + self.METRICS, ["status", "epoch"]) for _ in range(self.n_models)]
        self._controller = controller
        self._cluster_id = ipp_cluster_id
        self.active = 0
        self.lock = threading.RLock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.errors: List[str] = []
        self.listeners: List[Callable[[str, int], None]] = []    # UI refresh hooks

    # -- plumbing ----------------------------------------------------------------------
    @property
    def controller(self) -> ModelController:
        if self._controller is None:
            self._controller = ModelController(ipp_cluster_id=self._cluster_id)
        return self._controller

    def params_of(self, i: int) -> Dict[str, Any]:
        return {k: v[i] for k, v in self.compute_params.items()}

    def _notify(self, what: str, i: int) -> None:
        for fn in list(self.listeners):
            try:
                fn(what, i)
            except Exception as e:   # noqa: BLE001
                self.errors.append("listener failed: %r" % (e,))

    def _set(self, i: int, col: str, value) -> None:
        if col in self.table.columns:
            if self.table[col].dtype != object and not isinstance(value, (int, float, np.number)):
                self.table[col] = self.table[col].astype(object)
            self.table.at[i, col] = value

    # -- actions -----------------------------------------------------------------------
    def submit_computations(self, poll: bool = True, interval: float = 1.0) -> None:
        with self.lock:
            for i in range(self.n_models):
                self.controller.start_model(i, self.compute_func, self.params_of(i))
                self._set(i, "status", "Submitted")
        if poll:
            self.start_polling(interval)

    def stop_models(self, rows: Sequence[int], grace: Optional[float] = None) -> None:
        with self.lock:
            for i in rows:
                self.controller.stop_model(i, grace)
                self._set(i, "status", "Stopped")
                self._notify("row", i)

    def restart_models(self, rows: Sequence[int]) -> None:
        with self.lock:
            for i in rows:
                self.controller.restart_model(i, self.compute_func, self.params_of(i))
                self.data[i].reset()
                self._set(i, "status", "Restarted")
                self._set(i, "epoch", -1)
                for m in self.METRICS:
                    self._set(i, m, None)
                self.plots[i].update(self.data[i].get_plot_data())
                self._notify("row", i)

    def select(self, i: int) -> None:
        with self.lock:
            self.active = int(i)
            self.plots[i].update(self.data[i].get_plot_data())
            self._notify("select", i)

    # -- polling -------------------------------------------------------------------------
    def poll(self) -> int:
        """Apply every running trial's latest published data; returns rows changed."""
        changed = 0
        with self.lock:
            for i, fut in self.controller.get_running_models().items():
                data = fut.data
                done = fut.ready()
                if not data:
                    if done:
                        self._set(i, "status", "Done" if fut.successful() else "Failed")
                        self.controller.set_model_completed(i)
                        changed += 1
                        self._notify("row", i)
                    continue
                row_changed = False
                hist = data.get("history") or {}
                n_have = self.data[i].num_data_rows
                n_new = len(hist.get("epoch", []))
                if n_new > n_have:
                    for j in range(n_have, n_new):
                        self.data[i].append_plot_data_row({k: v[j] for k, v in hist.items() if j < len(v)})
                    for k, v in hist.items():
                        if v:
                            self._set(i, k, v[-1])
                    if i == self.active:
                        self.plots[i].update(self.data[i].get_plot_data())
                    row_changed = True
                if "status" in data:
                    self.data[i].set_status_data({"status": data["status"]})
                    self._set(i, "status", data["status"])
                    row_changed = True
                    if data["status"] == "Ended Training":
                        self.controller.set_model_completed(i)
                if "epoch" in data:
                    self.data[i].set_status_data({"epoch": data["epoch"]})
                    self._set(i, "epoch", data["epoch"])
                    row_changed = True
                if done:          # final data applied above; retire the future
                    if not fut.successful():
                        self._set(i, "status", "Failed")
                    self.controller.set_model_completed(i)
                    row_changed = True
                if row_changed:
                    changed += 1
                    self._notify("row", i)
        return changed

    def _loop(self, interval: float) -> None:
        while not self._stop.is_set():
            try:
                self.poll()
            except Exception as e:   # noqa: BLE001 - surfaced through .errors, loop keeps going
                self.errors.append("poll failed: %r" % (e,))
            if not self.controller.get_running_models():
                break
            self._stop.wait(interval)

    def start_polling(self, interval: float = 1.0) -> None:
        if self._thread is not None and self._thread.is_alive():
            return
        self._stop.clear()
        self._thread = threading.Thread(target=self._loop, args=(interval,), daemon=True, name="hpo-widget-poll")
        self._thread.start()

    def stop_polling(self, timeout: float = 5.0) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout)

    def wait(self, timeout: Optional[float] = None, interval: float = 0.2) -> bool:
        """Block until every trial has finished and its final data was applied."""
        t0 = time.time()
        while True:
            self.poll()
            if not self.controller.get_running_models():
                return True
            if timeout is not None and time.time() - t0 > timeout:
                return False
            time.sleep(interval)

    def get_models_status(self):
        with self.lock:
            return self.table[["status"]].copy()

    def resources_text(self) -> str:
        """Per-engine resource line for the dashboard: GPU, HBM in use / total, host RSS,
        queue depth and restarts (``get_resource_usage``)."""
        try:
            st = self.controller.get_resource_usage()
        except Exception:                # noqa: BLE001 - the dashboard must keep rendering
            return ""
        gib = lambda b: "%.2f" % (b / 2.0 ** 30)
        lines = []
        for eid in sorted(k for k in st if isinstance(k, int)):
            e = st[eid]
            hbm = ("HBM %s/%s GiB" % (gib(e["hbm_reserved_bytes"]), gib(e.get("hbm_total_bytes", 0)))
                   if "hbm_reserved_bytes" in e else "HBM -")
            rss = "RSS %s GiB" % gib(e["rss_bytes"]) if "rss_bytes" in e else "RSS -"
            lines.append("engine %d gpu %s: %s, %s, queue %d, restarts %d" % (
                eid, e.get("gpu"), hbm, rss, e.get("queue", 0), e.get("restarts", 0)))
        return "\n".join(lines)

    def snapshot(self):
        with self.lock:
            return copy.deepcopy(self.table)

    @property
    def results(self) -> List[Any]:
        """The trials' AsyncResults by row (running, completed or stopped) -- what the
        reference's analysis cells expect as ``psw.model_runs`` (``DistWidgetHPO_mnist.ipynb:
        269-280``, which referenced a missing attribute)."""
        return [self.controller.future(i) for i in range(self.n_models)]

    model_runs = results
