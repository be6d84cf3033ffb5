"""API-name aliases so the reference's notebooks and scripts run unchanged.

The reference imports Keras, Horovod, IPyParallel and Cray HPO by their own module
names (``mnist.py:15-21``, ``rpv.py:15-16,64``, ``train_rpv.py:10``, ``mlextras.py:3-6``,
``hpo_widgets.py:9``, ``CrayHPO_rpv.ipynb:44-45``).  ``install()`` registers this
framework's implementations under those names *when the real package is absent*:

    keras, keras.{layers,models,optimizers,callbacks,losses,utils,backend,datasets.mnist,
                  wrappers.scikit_learn}
    horovod, horovod.keras, horovod.keras.callbacks      -> parallel.hvd (RCCL data parallelism)
    ipyparallel, ipyparallel.datapub, ipyparallel.error  -> farm (one-node task farm)
    crayai, crayai.hpo, crayai.hpo.genetic               -> hpo (genetic search on GPU slots)

These are pure-Python name bindings onto the MI355X-native implementations -- no second
backend and no device-code shim.
"""
from __future__ import annotations

import importlib
import sys
import types
from typing import Dict


def _mod(name: str, doc: str = "", **attrs) -> types.ModuleType:
    m = types.ModuleType(name, doc)
    m.__dict__.update(attrs)
    return m


def _keras_modules() -> Dict[str, types.ModuleType]:
    from .. import losses as _losses
    from .. import models as _models
    from ..hpo import sklearn as _skl
    from ..models import layers as _layers
    from ..optim import optimizers as _opt
    from ..train import callbacks as _cb
    from .. import utils as _utils

    def set_image_data_format(fmt):
        if fmt != "channels_last":
            raise NotImplementedError("only channels_last is supported (the reference forces it, mnist.py:30)")

    def _mnist_load_data():
        """Keras' raw MNIST: ((x_train uint8 [N,28,28], y_train), (x_test, y_test))."""
        import numpy as np
        from ..apps.mnist import load_data
        xtr, ytr, xte, yte = load_data()
        to8 = lambda x: np.clip(np.rint(x[..., 0] * 255), 0, 255).astype(np.uint8)  # noqa: E731
        return (to8(xtr), ytr.argmax(1).astype(np.uint8)), (to8(xte), yte.argmax(1).astype(np.uint8))

    backend = _mod("keras.backend", "backend shims", set_image_data_format=set_image_data_format,
                   image_data_format=lambda: "channels_last", clear_session=_layers.reset_names,
                   epsilon=lambda: 1e-7, set_session=lambda s: None, get_session=lambda: None,
                   backend=lambda: "tensorflow", get_value=_opt.get_value, set_value=_opt.set_value)
    layers = _mod("keras.layers", **{k: getattr(_layers, k) for k in
                                     ("Input", "InputLayer", "Conv2D", "MaxPooling2D", "MaxPool2D", "Dropout",
                                      "Flatten", "Dense", "Layer") if hasattr(_layers, k)})
    if not hasattr(layers, "MaxPool2D"):
        layers.MaxPool2D = _layers.MaxPooling2D
    models = _mod("keras.models", Sequential=_models.Sequential, Model=_models.Model,
                  load_model=_models.load_model)
    utils = _mod("keras.utils", to_categorical=_utils.to_categorical)
    mnist = _mod("keras.datasets.mnist", load_data=_mnist_load_data)
    datasets = _mod("keras.datasets", mnist=mnist)
    scikit = _mod("keras.wrappers.scikit_learn", KerasClassifier=_skl.KerasClassifier,
                  KerasRegressor=_skl.KerasRegressor)
    wrappers = _mod("keras.wrappers", scikit_learn=scikit)
    keras = _mod("keras", "MI355X-native Keras-2.2-shaped API", __version__="2.2.4", layers=layers,
                 models=models, optimizers=_opt, callbacks=_cb, losses=_losses, utils=utils, backend=backend,
                 datasets=datasets, wrappers=wrappers, Sequential=_models.Sequential, Model=_models.Model)
    return {"keras": keras, "keras.layers": layers, "keras.models": models, "keras.optimizers": _opt,
            "keras.callbacks": _cb, "keras.losses": _losses, "keras.utils": utils, "keras.backend": backend,
            "keras.datasets": datasets, "keras.datasets.mnist": mnist, "keras.wrappers": wrappers,
            "keras.wrappers.scikit_learn": scikit}


def _horovod_modules() -> Dict[str, types.ModuleType]:
    from ..parallel import hvd
    horovod = _mod("horovod", keras=hvd)
    return {"horovod": horovod, "horovod.keras": hvd, "horovod.keras.callbacks": hvd.callbacks}


def _ipyparallel_modules() -> Dict[str, types.ModuleType]:
    from .. import farm
    from ..farm import magics
    from ..farm import protocol
    datapub = _mod("ipyparallel.datapub", publish_data=farm.publish_data)
    error = _mod("ipyparallel.error", RemoteError=protocol.RemoteError, CompositeError=protocol.RemoteError,
                 TaskAborted=protocol.TaskAborted, EngineError=protocol.EngineError)
    ipp = _mod("ipyparallel", "MI355X one-node task farm", __version__="6.2.0", Client=farm.Client,
               DirectView=farm.DirectView, LoadBalancedView=farm.LoadBalancedView, AsyncResult=farm.AsyncResult,
               datapub=datapub, error=error, RemoteError=protocol.RemoteError, px=magics.px)
    return {"ipyparallel": ipp, "ipyparallel.datapub": datapub, "ipyparallel.error": error}


def _crayai_modules() -> Dict[str, types.ModuleType]:
    from .. import hpo
    hmod = _mod("crayai.hpo", Params=hpo.Params, Evaluator=hpo.Evaluator, GeneticOptimizer=hpo.GeneticOptimizer,
                genetic=hpo.genetic, __version__="0.4.0")
    return {"crayai": _mod("crayai", hpo=hmod), "crayai.hpo": hmod, "crayai.hpo.genetic": hpo.genetic}


_GROUPS = {"keras": _keras_modules, "horovod": _horovod_modules, "ipyparallel": _ipyparallel_modules,
           "crayai": _crayai_modules}


def _importable(name: str) -> bool:
    if name in sys.modules:
        return True
    try:
        return importlib.util.find_spec(name) is not None
    except (ImportError, ValueError):
        return False


def install(force: bool = False, groups=("keras", "horovod", "ipyparallel", "crayai")) -> Dict[str, str]:
    """Register the aliases; returns ``{top-level name: 'installed' | 'present'}``."""
    out = {}
    for g in groups:
        if not force and _importable(g) and not getattr(sys.modules.get(g), "__intml_alias__", False):
            out[g] = "present"
            continue
        mods = _GROUPS[g]()
        for name, m in mods.items():
            try:
                m.__intml_alias__ = True
            except AttributeError:
                pass
            sys.modules[name] = m
        out[g] = "installed"
    return out
