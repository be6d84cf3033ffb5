"""Notebook rendering of the HPO dashboard (``hpo_widgets.py`` call shapes):

    plot = partial(ModelPlot, y=['loss', 'acc', 'val_loss', 'val_acc'], xlim=[0, n_epochs])
    psw = ParamSpanWidget(build_and_train, plot, params, ipp_cluster_id=cluster_id)
    display(psw); psw.submit_computations()                 # DistWidgetHPO_mnist.ipynb:225-252

With ipywidgets + bqplot installed the widgets are live (table via qgrid if present,
else an HTML table; Stop/Restart buttons act on the selected rows).  Without them --
as in this image, where none of the widget stack is installed -- the same classes work
headless: they keep the full state (``widgets/model.py``) and render as text
(``render()``), so scripts and tests drive exactly the same logic.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional, Sequence

from .model import ModelController, ParamSpanModel, PlotModel

try:      # optional UI stack
    import bqplot as _bq
    import ipywidgets as _ipw
    HAVE_WIDGETS = True
except Exception:       # noqa: BLE001
    _bq = _ipw = None
    HAVE_WIDGETS = False

try:
    import qgrid as _qgrid
except Exception:       # noqa: BLE001
    _qgrid = None


def _text_table(df) -> str:
    try:
        return df.to_string()
    except Exception:       # noqa: BLE001
        return str(df)


if HAVE_WIDGETS:
    class ModelPlot(_ipw.VBox):
        COLORS = ["blue", "red", "green", "orange", "black", "purple", "gray"]

        def __init__(self, y, x=None, xlim=None, ylim=None, xlabel=None, ylabel=None, title=None):
            super().__init__()
            self.model = PlotModel(y, x, xlim, ylim, xlabel, ylabel, title)
            m = self.model
            self.xscale = _bq.LinearScale(min=m.xlim[0], max=m.xlim[1])
            self.yscale = _bq.LinearScale(min=m.ylim[0], max=m.ylim[1])
            axes = [_bq.Axis(scale=self.xscale, label=m.xlabel, grid_lines="none"),
                    _bq.Axis(scale=self.yscale, label=m.ylabel if isinstance(m.ylabel, str) else "",
                             orientation="vertical", grid_lines="none")]
            self.lines, self.scatters = [], []
            for k, name in enumerate(m.y):
                color = self.COLORS[k % len(self.COLORS)]
                sc = {"x": self.xscale, "y": self.yscale}
                self.lines.append(_bq.Lines(x=[], y=[], scales=sc, colors=[color], labels=[name],
                                            display_legend=len(m.y) > 1, enable_hover=True))
                self.scatters.append(_bq.Scatter(x=[], y=[], scales=sc, colors=[color], enable_hover=True))
            self.fig = _bq.Figure(marks=self.lines + self.scatters, axes=axes, title=m.title,
                                  layout=_ipw.Layout(height="550px", width="100%"))
            self.children = [self.fig]

        @property
        def y(self):
            return self.model.y

        def update(self, data):
            self.model.update(data)
            for k, name in enumerate(self.model.y):
                s = self.model.series[name]
                for mark in (self.lines[k], self.scatters[k]):
                    mark.x, mark.y = s["x"], s["y"]
            self.xscale.min, self.xscale.max = self.model.xlim
            self.yscale.min, self.yscale.max = self.model.ylim

    class ParamSpanWidget(_ipw.VBox):
        def __init__(self, compute_func, vis_func, params, columns=None, ipp_cluster_id=None,
                      output_layout=None, qgrid_layout=None, controller=None):
            super().__init__()
            self.model = ParamSpanModel(compute_func, params, vis_func=vis_func, controller=controller,
                                        ipp_cluster_id=ipp_cluster_id, columns=columns)
            self.output = _ipw.Output(layout=output_layout or _ipw.Layout(height="600px", border="1px solid",
                                                                          overflow_y="scroll"))
            self.debug = _ipw.Output()
            if _qgrid is not None:
                self.table = _qgrid.QGridWidget(df=self.model.table, layout=qgrid_layout or _ipw.Layout())
                self.table.grid_options.update(editable=False, forceFitColumns=True, defaultColumnWidth=200)
                self.table.on("selection_changed", lambda ev, w: ev["new"] and self.model.select(ev["new"][0]))
            else:
                self.table = _ipw.HTML()
                self.selector = _ipw.Dropdown(options=list(range(self.model.n_models)), description="model")
                self.selector.observe(lambda ch: self.model.select(ch["new"]), names="value")
            stop, restart = _ipw.Button(description="Stop selected"), _ipw.Button(description="Restart selected")
            stop.on_click(lambda _: self.model.stop_models(self.selected_rows()))
            restart.on_click(lambda _: self.model.restart_models(self.selected_rows()))
            extra = [] if _qgrid is not None else [self.selector]
            self.children = [self.output, _ipw.HBox(extra + [stop, restart]), self.table]
            self.model.listeners.append(self._on_change)
            self.model.select(0)

        def selected_rows(self):
            if _qgrid is not None:
                return list(self.table.get_selected_rows())
            return [self.selector.value]

        def _on_change(self, what, i):
            if _qgrid is not None:
                self.table.df = self.model.snapshot()
            else:
                self.table.value = self.model.snapshot().to_html()
            if what == "select" or i == self.model.active:
                from IPython.display import clear_output, display
                with self.output:
                    clear_output(wait=True)
                    display(self.model.plots[self.model.active])

        def submit_computations(self, interval=1.0):
            self.model.submit_computations(poll=True, interval=interval)

        def __getattr__(self, item):     # expose the headless model's API
            return getattr(self.__dict__["model"], item) if "model" in self.__dict__ else \
                super().__getattribute__(item)

else:
    class ModelPlot(PlotModel):
        """Headless ModelPlot: same constructor and ``update(data)``; ``render()`` gives text."""

        def render(self) -> str:
            lines = [self.title]
            for k, s in self.series.items():
                pts = ", ".join("%g:%.4f" % (x, y) for x, y in zip(s["x"], s["y"]))
                lines.append("  %s: %s" % (k, pts))
            return "\n".join(lines)

        def __repr__(self):
            return self.render()

    class ParamSpanWidget(ParamSpanModel):
        """Headless ParamSpanWidget with the reference's constructor signature."""

        def __init__(self, compute_func: Callable, vis_func: Optional[Callable], params: Dict[str, Sequence],
                     columns=None, ipp_cluster_id=None, output_layout=None, qgrid_layout=None,
                     controller: Optional[ModelController] = None):
            super().__init__(compute_func, params, vis_func=vis_func, controller=controller,
                             ipp_cluster_id=ipp_cluster_id, columns=columns)

        def stop_selected_models(self, rows: Sequence[int] = None):
            self.stop_models(rows if rows is not None else [self.active])

        def restart_selected_models(self, rows: Sequence[int] = None):
            self.restart_models(rows if rows is not None else [self.active])

        def render(self) -> str:
            with self.lock:
                out = _text_table(self.table) + "\n\n" + self.plots[self.active].render() \
                    if hasattr(self.plots[self.active], "render") else _text_table(self.table)
            res = self.resources_text()
            return out + ("\n\n" + res if res else "")

        def __repr__(self):
            return self.render()
