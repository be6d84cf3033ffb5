"""``from hpo_widgets import ModelPlot, ParamSpanWidget`` (live HPO dashboard)."""
import _path  # noqa: F401
from cori_intml_examples_amd.widgets import (ModelController, ModelPlot, ModelPlotTable,  # noqa: F401
                                             ModelTaskData, ParamSpanWidget)
