"""Keras-2.2-compatible HDF5 checkpoints: ``save_model`` / ``load_model`` /
``save_weights`` / ``load_weights``.

Reference call sites: ``ModelCheckpoint(checkpoint_file)`` writes the whole model every
epoch (``rpv.py:100-101``; ``model_%i.h5`` per trial at ``DistHPO_mnist.ipynb:184-185,248``)
and ``keras.models.load_model(file)`` reloads the best trial for test evaluation
(``DistHPO_mnist.ipynb:540-542``, ``DistHPO_rpv.ipynb:397-399``).

File layout, written through the native ``_h5lite`` module:

    /                       attrs keras_version, backend, model_config (JSON), training_config (JSON)
    /model_weights          attrs layer_names, backend, keras_version
    /model_weights/<layer>  attr  weight_names = ["<layer>/kernel:0", "<layer>/bias:0"]
    /model_weights/<layer>/<layer>/kernel:0   (kh,kw,Cin,Cout) | (in,out) float32
    /optimizer_weights      attr  weight_names; one dataset per optimizer variable

Optimizer variables follow Keras 2.2.4's ``Optimizer.weights`` order:
Adam ``[iterations] + m + v + vhat``, Nadam ``[iterations] + m + v``, Adadelta
``accumulators + delta_accumulators``, RMSprop ``accumulators``, SGD ``[iterations] + moments``.
The DistributedOptimizer wrapper serialises under its base class name so the file
reloads without the parallel package (Appendix B.2 last bullet).  Writes go to a
temporary file that is renamed into place, so a crash mid-save never leaves a torn
checkpoint (ModelCheckpoint overwrites one file per epoch).
"""
from __future__ import annotations

import json
import os
from typing import List, Optional

import numpy as np

from .h5 import H5File

KERAS_VERSION = "2.2.4"


# ----------------------------------------------------------------------------- helpers
def _weighted_layers(model):
    return [l for l in model.layers]


def _layer_weight_names(layer) -> List[str]:
    return ["%s/%s:0" % (layer.name, n) for n, _, _ in layer.weight_specs()]


def _loss_name(loss):
    if isinstance(loss, str) or loss is None:
        return loss
    return getattr(loss, "__name__", str(loss))


def _opt_layout(opt, n_params):
    """[(name, source)] where source is ('iter',) | ('slot', k, param_index) | ('zero1', i)."""
    cls = type(opt).__name__
    out = []
    if cls == "Adam":
        out.append(("Adam/iterations:0", ("iter",)))
        for k in (0, 1):
            for i in range(n_params):
                out.append((None, ("slot", k, i)))
        for i in range(n_params):
            out.append((None, ("zero1", i)))
    elif cls == "Nadam":
        out.append(("Nadam/iterations:0", ("iter",)))
        for k in (0, 1):
            for i in range(n_params):
                out.append((None, ("slot", k, i)))
    elif cls == "Adadelta":
        for k in (0, 1):
            for i in range(n_params):
                out.append((None, ("slot", k, i)))
    elif cls == "RMSprop":
        for i in range(n_params):
            out.append((None, ("slot", 0, i)))
    else:   # SGD
        out.append(("SGD/iterations:0", ("iter",)))
        for i in range(n_params):
            out.append((None, ("slot", 0, i)))
    # Keras names the unnamed slot variables training/<Opt>/Variable[_k]:0 in creation order
    named, j = [], 0
    for name, src in out:
        if name is None:
            name = "training/%s/Variable%s:0" % (cls, "" if j == 0 else "_%d" % j)
            j += 1
        named.append((name, src))
    return named


def _param_specs(model):
    return list(model.store.specs) if model.store is not None else []


# ----------------------------------------------------------------------------- save
def _write_weights(f: H5File, model, group: str = "model_weights") -> None:
    f.create_group(group)
    layers = _weighted_layers(model)
    a = f.attrs(group)
    a["layer_names"] = [l.name for l in layers]
    a["backend"] = "tensorflow"
    a["keras_version"] = KERAS_VERSION
    for layer in layers:
        g = group.rstrip("/") + "/" + layer.name
        f.create_group(g)
        names = _layer_weight_names(layer)
        f.attrs(g)["weight_names"] = names
        for name, value in zip(names, layer.get_weights()):
            f.write_dataset(g + "/" + name, np.ascontiguousarray(value, dtype=np.float32))


def _write_optimizer(f: H5File, model) -> None:
    ex = model._executor
    opt = getattr(model.optimizer, "_base_optimizer", model.optimizer)
    if ex is None or opt is None:
        return
    specs = _param_specs(model)
    slots = [s.detach().float().cpu().numpy() for s in ex.optimizer_state()]
    layout = _opt_layout(opt, len(specs))
    f.create_group("optimizer_weights")
    f.attrs("optimizer_weights")["weight_names"] = [n for n, _ in layout]
    for name, src in layout:
        if src[0] == "iter":
            val = np.asarray(opt.iterations, dtype=np.int64)
        elif src[0] == "zero1":
            val = np.zeros((1,), np.float32)
        else:
            k, i = src[1], src[2]
            s = specs[i]
            val = (slots[k][s.offset:s.offset + s.numel].reshape(s.shape) if k < len(slots)
                   else np.zeros(s.shape, np.float32))
        f.write_dataset("optimizer_weights/" + name, np.ascontiguousarray(val))
    # not part of Keras' file (it keeps Nadam's m_schedule out of the weights), stored so
    # a resumed Nadam run continues bit-identically; ignored by Keras readers
    f.attrs("optimizer_weights")["intml_iterations"] = np.asarray(opt.iterations, dtype=np.int64)
    ms = getattr(ex, "m_schedule_value", None)
    if callable(ms):
        f.attrs("optimizer_weights")["intml_m_schedule"] = np.asarray(ms(), dtype=np.float64)


def _atomic_target(filepath: str) -> str:
    d = os.path.dirname(os.path.abspath(filepath))
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, ".%s.tmp%d" % (os.path.basename(filepath), os.getpid()))


def save_model(model, filepath: str, overwrite: bool = True, include_optimizer: bool = True) -> None:
    filepath = str(filepath)
    if not overwrite and os.path.exists(filepath):
        raise FileExistsError(filepath)
    tmp = _atomic_target(filepath)
    try:
        with H5File(tmp, "w") as f:
            a = f.attrs("/")
            a["keras_version"] = KERAS_VERSION
            a["backend"] = "tensorflow"
            a["model_config"] = json.dumps({"class_name": type(model).__name__ if type(model).__name__ in
                                            ("Sequential", "Model") else "Model",
                                            "config": model.get_config()})
            _write_weights(f, model)
            if include_optimizer and model.optimizer is not None and model._compiled:
                from ..optim import optimizers
                a["training_config"] = json.dumps({
                    "optimizer_config": optimizers.serialize(model.optimizer),
                    "loss": _loss_name(model.loss), "metrics": list(model.metrics),
                    "sample_weight_mode": None, "loss_weights": None})
                _write_optimizer(f, model)
        os.replace(tmp, filepath)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def save_weights(model, filepath: str) -> None:
    tmp = _atomic_target(str(filepath))
    try:
        with H5File(tmp, "w") as f:
            _write_weights(f, model, "/")
        os.replace(tmp, str(filepath))
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


# ----------------------------------------------------------------------------- load
def _read_weights(f: H5File, model, group: str) -> None:
    names = f.attrs(group)["layer_names"]
    by_name = {l.name: l for l in model.layers}
    weighted = [l for l in model.layers if l.weight_specs()]
    stored = [n for n in names if f.attrs(group + "/" + n if group != "/" else "/" + n).get("weight_names", [])]
    if len(stored) != len(weighted):
        raise ValueError("checkpoint has %d layers with weights, model has %d" % (len(stored), len(weighted)))
    values = []
    for lname, layer in zip(stored, weighted):
        g = (group.rstrip("/") + "/" + lname) if group != "/" else "/" + lname
        wn = f.attrs(g)["weight_names"]
        values.extend(f.read_dataset(g + "/" + w) for w in wn)
    del by_name
    model.store.set_weights(values)
    model._weights_changed()


def load_weights(model, filepath: str) -> None:
    with H5File(str(filepath), "r") as f:
        group = "model_weights" if "model_weights" in f else "/"
        _read_weights(f, model, group)


def model_from_config(config: dict, device=None):
    from ..models.layers import LAYER_CLASSES, InputLayer
    from ..models.model import Model, Sequential
    cls, cfg = config["class_name"], config["config"]
    if cls == "Sequential":
        layer_cfgs = cfg["layers"] if isinstance(cfg, dict) else cfg
        name = cfg.get("name") if isinstance(cfg, dict) else None
        model = Sequential(name=name, device=device)
        for lc in layer_cfgs:
            model.add(LAYER_CLASSES[lc["class_name"]].from_config(lc["config"]))
        return model
    if cls == "Model":
        layers = {}
        order = cfg["layers"]
        for lc in order:
            layers[lc["name"]] = LAYER_CLASSES[lc["class_name"]].from_config(lc["config"])
        from ..models.layers import KTensor
        tensors = {}
        for lc in order:
            layer = layers[lc["name"]]
            if isinstance(layer, InputLayer):
                tensors[lc["name"]] = KTensor(layer.output_shape_, layer, None)
            else:
                inbound = lc["inbound_nodes"][0][0][0]
                tensors[lc["name"]] = layer(tensors[inbound])
        inp = tensors[cfg["input_layers"][0][0]]
        out = tensors[cfg["output_layers"][0][0]]
        return Model(inputs=inp, outputs=out, name=cfg.get("name"), device=device)
    raise ValueError("unknown model class %r" % cls)


def load_model(filepath: str, custom_objects=None, compile: bool = True, device=None):
    from ..optim import optimizers
    with H5File(str(filepath), "r") as f:
        root = f.attrs("/")
        model = model_from_config(json.loads(root["model_config"]), device=device)
        _read_weights(f, model, "model_weights")
        tc = root.get("training_config")
        if compile and tc:
            tc = json.loads(tc)
            opt = optimizers.deserialize(tc["optimizer_config"])
            model.compile(optimizer=opt, loss=tc["loss"], metrics=tc.get("metrics") or None)
            if "optimizer_weights" in f:
                names = f.attrs("optimizer_weights")["weight_names"]
                vals = [f.read_dataset("optimizer_weights/" + n) for n in names]
                it = f.attrs("optimizer_weights").get("intml_iterations")
                _restore_optimizer(model, opt, vals, None if it is None else int(it))
                ms = f.attrs("optimizer_weights").get("intml_m_schedule")
                if ms is not None and hasattr(model._executor, "set_m_schedule"):
                    model._executor.set_m_schedule(float(ms))
    return model


def _restore_optimizer(model, opt, vals, iterations_hint=None) -> None:
    specs = _param_specs(model)
    layout = _opt_layout(opt, len(specs))
    if len(layout) != len(vals):
        raise ValueError("optimizer_weights has %d entries, %s expects %d" % (len(vals), type(opt).__name__,
                                                                             len(layout)))
    n_slots = getattr(opt, "n_slots", 0)
    numel = model.store.numel
    slots = [np.zeros(numel, np.float32) for _ in range(n_slots)]
    iterations = 0
    for (name, src), v in zip(layout, vals):
        if src[0] == "iter":
            iterations = int(np.asarray(v).reshape(-1)[0])
        elif src[0] == "slot" and src[1] < n_slots:
            s = specs[src[2]]
            slots[src[1]][s.offset:s.offset + s.numel] = np.asarray(v, np.float32).reshape(-1)
    if iterations_hint is not None:
        iterations = iterations_hint
    elif type(opt).__name__ in ("Adadelta", "RMSprop"):
        iterations = 0      # Keras does not store the counter for these
    model._executor.set_optimizer_state(iterations, slots)
