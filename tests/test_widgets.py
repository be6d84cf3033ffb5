"""Headless HPO dashboard (SURVEY.md §4.3 "Widget tests"): drive ModelTaskData /
ModelPlotTable / ParamSpanModel with synthetic publish events and assert table and plot
state; then one run against CPU farm engines with working Stop / Restart."""
import os
import sys
import time

import cloudpickle
import numpy as np
import pytest

from cori_intml_examples_amd.widgets import (ModelController, ModelPlot, ModelPlotTable, ModelTaskData,
                                             ParamSpanModel, ParamSpanWidget, PlotModel)

cloudpickle.register_pickle_by_value(sys.modules[__name__])


def test_plot_table_and_task_data():
    t = ModelPlotTable(["epoch", "loss"])
    t.append_row({"epoch": 0, "loss": 1.0})
    t.append_row({"epoch": 1})
    assert t.to_dict() == {"epoch": [0, 1], "loss": [1.0, None]}
    t.append_column("acc")
    assert t.to_dict()["acc"] == [None, None] and t.columns == ["epoch", "loss", "acc"]
    with pytest.raises(KeyError):
        t.append_column("acc")
    with pytest.raises(ValueError):
        t.append_column("x", [1])
    # a valued column after a value-less one lands under its own name
    t.append_column("f1", [0.3, 0.4])
    assert t.to_dict()["acc"] == [None, None] and t.to_dict()["f1"] == [0.3, 0.4]
    t.append_row({"epoch": 2, "acc": 0.9, "f1": 0.5})
    assert t.column("acc") == [None, None, 0.9] and t.column("f1") == [0.3, 0.4, 0.5]
    d = ModelTaskData(["epoch", "loss"], ["status", "epoch"])
    assert d.num_data_rows == 0 and d.has_updates
    d.append_plot_data_row({"epoch": 0, "loss": 0.5})
    d.set_status_data({"status": "Begin Epoch"})
    assert d.num_data_rows == 1 and d.get_status_data()["status"] == "Begin Epoch"


def test_plot_model_extents():
    p = PlotModel(["loss", "acc"], x="epoch", xlim=[0, 4])
    p.update({"epoch": [0, 1, 2], "loss": [2.5, 1.0, 0.5], "acc": [0.1, 0.5, 0.9]})
    assert p.num_points == 3 and p.ylim == [0, 2.5] and p.xlim == [0, 4]
    np.testing.assert_array_equal(p.series["acc"]["y"], [0.1, 0.5, 0.9])
    p.update({"loss": [1.0]})                   # no x column -> index
    np.testing.assert_array_equal(p.series["loss"]["x"], [0])
    assert isinstance(ModelPlot(["loss"], title="t"), object)


class _FakeFuture:
    def __init__(self):
        self.data = {}
        self._done = False
        self._ok = True
        self.aborted = False

    def ready(self):
        return self._done

    done = ready

    def successful(self):
        return self._ok

    def abort(self, grace=None):
        self.aborted = True
        self._done, self._ok = True, False


class _FakeView:
    def __init__(self):
        self.submitted = []

    def apply(self, f, **kw):
        fut = _FakeFuture()
        self.submitted.append((kw, fut))
        return fut


def _publish(fut, status, epoch=None, n=0):
    hist = {"loss": [1.0 / (i + 1) for i in range(n)], "acc": [0.5 + 0.1 * i for i in range(n)],
            "val_loss": [1.1 / (i + 1) for i in range(n)], "val_acc": [0.4 + 0.1 * i for i in range(n)],
            "epoch": list(range(n))}
    fut.data = {"status": status, "history": hist}
    if epoch is not None:
        fut.data["epoch"] = epoch


def test_param_span_model_with_synthetic_events():
    view = _FakeView()
    ctl = ModelController(view=view)
    params = {"h1": [4, 8, 16], "dropout": [0.1, 0.2, 0.3], "conv": [[1, 2], [3, 4], [5, 6]]}
    m = ParamSpanModel(lambda **kw: None, params, controller=ctl)
    assert list(m.table.columns) == ["status", "epoch", "h1", "dropout", "conv", "loss", "val_loss", "acc", "val_acc"]
    assert m.table.conv[0] == "[1, 2]" and (m.table.status == "Not Started").all()
    m.submit_computations(poll=False)
    assert [kw for kw, _ in view.submitted][1] == {"h1": 8, "dropout": 0.2, "conv": [3, 4]}
    f0, f1, f2 = [f for _, f in view.submitted]
    _publish(f0, "Begin Training")
    _publish(f1, "Ended Epoch", epoch=1, n=2)
    assert m.poll() == 2
    assert m.table.status[0] == "Begin Training" and m.table.epoch[1] == 1
    assert m.table.val_acc[1] == pytest.approx(0.5) and m.data[1].num_data_rows == 2
    _publish(f1, "Ended Epoch", epoch=2, n=3)
    m.poll()
    assert m.data[1].num_data_rows == 3                # appended exactly once each
    assert m.data[1].get_plot_data()["epoch"] == [0, 1, 2]
    m.select(1)
    assert m.plots[1].num_points == 3
    # completion, failure, stop, restart
    _publish(f1, "Ended Training", n=3)
    f1._done = True
    f2._done, f2._ok = True, False
    m.poll()
    assert m.table.status[1] == "Ended Training" and m.table.status[2] == "Failed"
    assert set(ctl.get_running_models()) == {0}
    m.stop_models([0])
    assert f0.aborted and m.table.status[0] == "Stopped" and ctl.get_running_models() == {}
    m.restart_models([0])
    assert len(view.submitted) == 4 and m.table.status[0] == "Restarted" and m.data[0].num_data_rows == 0
    assert "Restarted" in m.get_models_status().status.tolist()


def _trial(lr, n_epochs=3, sleep=0.05):
    from cori_intml_examples_amd.farm import publish_data, should_stop
    hist = {"acc": [], "loss": [], "val_acc": [], "val_loss": [], "epoch": []}
    publish_data({"status": "Begin Training", "history": hist})
    for e in range(n_epochs):
        for _ in range(int(1 + sleep / 0.01)):
            time.sleep(0.01)
            if should_stop():
                return "stopped"
        for k in ("acc", "loss", "val_acc", "val_loss"):
            hist[k].append(lr * (e + 1))
        hist["epoch"].append(e)
        publish_data({"status": "Ended Epoch", "epoch": e, "history": hist})
    publish_data({"status": "Ended Training", "history": hist})
    return hist


def test_widget_on_farm_with_stop_restart():
    from functools import partial

    from cori_intml_examples_amd import farm
    cl = farm.start_cluster(2, cluster_id="pytest_w_%d" % os.getpid(), cpu_only=True, abort_grace=2.0)
    try:
        with cl.client() as c:
            ctl = ModelController(client=c)
            plot = partial(ModelPlot, y=["loss", "acc", "val_loss", "val_acc"], x="epoch", xlim=[0, 3])
            psw = ParamSpanWidget(partial(_trial, n_epochs=3), plot, {"lr": [0.1, 0.2, 0.3]}, controller=ctl)
            psw.submit_computations(poll=False)
            assert psw.wait(timeout=120)
            assert (psw.table.status == "Ended Training").all()
            assert psw.table.epoch.tolist() == [2, 2, 2]
            assert psw.data[2].get_plot_data()["loss"] == pytest.approx([0.3, 0.6, 0.9])
            assert "lr" in psw.render()
            # stop a long trial, then restart it with the same parameters
            slow = ParamSpanWidget(partial(_trial, n_epochs=3, sleep=5.0), plot, {"lr": [0.5]}, controller=ctl)
            slow.submit_computations(poll=False)
            time.sleep(1.0)
            slow.stop_selected_models([0])
            assert slow.table.status[0] == "Stopped"
            fut = ctl._stopped[0]
            assert fut.wait(30) and fut.get(5) == "stopped"        # cooperative stop honoured
            slow.restart_selected_models([0])
            assert ctl.get_running_models()[0] is not fut
            ctl.stop_model(0, grace=0.5)
    finally:
        cl.stop()
