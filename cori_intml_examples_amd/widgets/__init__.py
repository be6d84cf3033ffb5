"""Live HPO monitoring widgets (``hpo_widgets.py``): a headless, testable data model plus
an ipywidgets/bqplot front-end when that stack is installed."""
from .model import ModelController, ModelPlotTable, ModelTaskData, ParamSpanModel, PlotModel
from .ui import HAVE_WIDGETS, ModelPlot, ParamSpanWidget

__all__ = ["ModelPlot", "ParamSpanWidget", "ModelController", "ModelTaskData", "ModelPlotTable",
           "ParamSpanModel", "PlotModel", "HAVE_WIDGETS"]
