"""Keras-2.2-shaped ``Model`` / ``Sequential``.

Call shapes that must work: ``Sequential().add(...)`` (``mnist.py:47-56``),
functional ``Model(inputs, outputs, name)`` (``rpv.py:68``), ``compile(optimizer=str|obj,
loss=str|fn, metrics=['accuracy'])``, ``fit(..., validation_data | validation_split,
callbacks, verbose)`` -> History, ``evaluate``, ``predict``, ``predict_classes``,
``summary()`` in Keras table format, ``save`` / ``models.load_model``.

Execution is delegated to an executor: the HIP/gfx950 backend when the model lives on
a GPU (graph-captured fused step), the CPU reference backend otherwise.
"""
from __future__ import annotations

import sys
import time
from typing import List, Optional

import numpy as np
import torch

from .. import optim as optimizers
from ..train import callbacks as cbks
from ..utils.env import default_device, next_seed
from .executor_base import DeviceData
from .layers import Dense, InputLayer, KTensor, Layer
from .params import ParamStore
from .plan import build_plan, canonical_loss


def _norm_device(device) -> torch.device:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


class Model:
    def __init__(self, inputs=None, outputs=None, name=None, device=None):
        self.name = name or type(self).__name__.lower()
        self._chain: List[Layer] = []        # InputLayer first
        self.store: Optional[ParamStore] = None
        self.optimizer = None
        self.loss = None
        self.metrics = []
        self._executor = None
        self._plan = None
        self.stop_training = False
        self.history = None
        self._device = _norm_device(device) if device is not None else None
        self._seed = next_seed()
        self._compiled = False
        if inputs is not None or outputs is not None:
            self._init_graph(inputs, outputs)

    # ------------------------------------------------------------------ graph construction
    def _init_graph(self, inputs, outputs):
        if isinstance(inputs, (list, tuple)):
            if len(inputs) != 1:
                raise NotImplementedError("multi-input models")
            inputs = inputs[0]
        if isinstance(outputs, (list, tuple)):
            if len(outputs) != 1:
                raise NotImplementedError("multi-output models")
            outputs = outputs[0]
        chain = []
        t = outputs
        while t is not None:
            chain.append(t.layer)
            t = t.inbound
        chain.reverse()
        if chain[0] is not inputs.layer:
            raise ValueError("outputs are not connected to inputs")
        self._chain = chain
        self._build_store()

    def _build_store(self):
        for layer in self._chain:
            layer.model = self
        self._device = self._device or _norm_device(default_device())
        self.store = ParamStore(self._chain, self._device)
        self.store.initialize(self._seed)

    @property
    def layers(self) -> List[Layer]:
        return list(self._chain)

    @property
    def inputs(self):
        return [self._chain[0]] if self._chain else []

    @property
    def input_shape(self):
        return self._chain[0].output_shape if self._chain else None

    @property
    def output_shape(self):
        return self._chain[-1].output_shape if self._chain else None

    @property
    def device(self):
        return self._device

    def get_layer(self, name=None, index=None):
        if index is not None:
            return self.layers[index]
        for layer in self.layers:
            if layer.name == name:
                return layer
        raise ValueError("No such layer: %s" % name)

    def to(self, device) -> "Model":
        """Move the model (weights) to another device; optimizer state is reset."""
        device = torch.device(device)
        weights = self.get_weights() if self.store is not None else None
        self._device = device
        if self._chain:
            self._build_store()
            if weights is not None:
                self.store.set_weights(weights)
        if self._compiled:
            self._make_executor()
        return self

    # ------------------------------------------------------------------ weights
    def count_params(self) -> int:
        return sum(l.count_params() for l in self._chain)

    def get_weights(self):
        return self.store.get_weights() if self.store else []

    def set_weights(self, weights):
        self.store.set_weights(weights)
        self._weights_changed()

    def _weights_changed(self):
        if self._executor is not None:
            self._executor.params_changed()

    @property
    def weights(self):
        return [w for l in self._chain for w in l.weights]

    # ------------------------------------------------------------------ compile
    def compile(self, optimizer, loss=None, metrics=None, loss_weights=None, sample_weight_mode=None,
                **kwargs):
        if not self._chain:
            raise RuntimeError("model has no layers")
        if loss_weights is not None or sample_weight_mode is not None:
            raise NotImplementedError("loss_weights / sample_weight_mode")
        self.optimizer = optimizers.get(optimizer)
        self.loss = loss
        canonical_loss(loss)
        self.metrics = list(metrics or [])
        for m in self.metrics:
            if m not in ("accuracy", "acc"):
                raise NotImplementedError("metric %r" % (m,))
        self._plan = build_plan(self._chain, loss)
        self._compiled = True
        self._make_executor()

    def _make_executor(self):
        base = getattr(self.optimizer, "_base_optimizer", self.optimizer)
        if self._device.type == "cuda":
            from .executor_hip import HipExecutor
            self._executor = HipExecutor(self._plan, self.store, base, self._seed)
        else:
            from .executor_ref import RefExecutor
            self._executor = RefExecutor(self._plan, self.store, base, self._seed)
        if getattr(self.optimizer, "distributed", False):
            from ..parallel import dist
            self._executor.reducer = dist.make_reducer(self._executor, self.optimizer)

    @property
    def metrics_names(self):
        return ["loss"] + (["acc"] if self.metrics else [])

    def _check_compiled(self):
        if not self._compiled:
            raise RuntimeError("You must compile your model before using it.")

    # ------------------------------------------------------------------ training
    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose=1, callbacks=None,
            validation_split=0.0, validation_data=None, shuffle=True, class_weight=None,
            sample_weight=None, initial_epoch=0, steps_per_epoch=None, validation_steps=None,
            **kwargs):
        from ..train.loop import fit_loop
        self._check_compiled()
        if class_weight is not None or sample_weight is not None:
            raise NotImplementedError("class_weight / sample_weight in fit")
        if steps_per_epoch is not None:
            raise NotImplementedError("steps_per_epoch")
        return fit_loop(self, x, y, batch_size or 32, epochs, verbose, callbacks, validation_split,
                        validation_data, shuffle, initial_epoch)

    def evaluate(self, x=None, y=None, batch_size=None, verbose=1, sample_weight=None, steps=None):
        self._check_compiled()
        ex = self._executor
        data = x if isinstance(x, DeviceData) else ex.upload(x, y)
        self._run_eval(data, batch_size or 32)
        loss, acc, _ = ex.read_metrics()
        if verbose:
            print("%d/%d [==============================] - loss: %.4f%s" % (
                data.n, data.n, loss, (" - acc: %.4f" % acc) if self.metrics else ""))
        return [loss, acc] if self.metrics else loss

    def _run_eval(self, data, batch_size):
        ex = self._executor
        ex.reset_metrics()
        pos = 0
        while pos < data.n:
            bs = min(batch_size, data.n - pos)
            ex.eval_step(data, pos, bs)
            pos += bs

    def predict(self, x, batch_size=None, verbose=0, steps=None):
        self._check_compiled_or_plan()
        ex = self._executor
        data = ex.upload(x, None)
        batch_size = batch_size or 32
        outs = []
        pos = 0
        while pos < data.n:
            bs = min(batch_size, data.n - pos)
            outs.append(ex.predict_step(data, pos, bs).float().cpu())
            pos += bs
        return torch.cat(outs).numpy() if outs else np.zeros((0,) + tuple(self.output_shape[1:]))

    def _check_compiled_or_plan(self):
        if self._executor is None:
            # Keras allows predict() on an uncompiled model: compile a throw-away executor
            self._plan = build_plan(self._chain, "mse" if self._chain[-1].activation is None else (
                "binary_crossentropy" if self._chain[-1].activation == "sigmoid"
                else "categorical_crossentropy"))
            self.optimizer = self.optimizer or optimizers.SGD()
            self._make_executor()

    def predict_proba(self, x, batch_size=32, verbose=0):
        return self.predict(x, batch_size, verbose)

    def predict_classes(self, x, batch_size=32, verbose=0):
        p = self.predict(x, batch_size, verbose)
        if p.shape[-1] > 1:
            return p.argmax(axis=-1)
        return (p > 0.5).astype("int32")

    def train_on_batch(self, x, y):
        self._check_compiled()
        ex = self._executor
        data = ex.upload(x, y)
        ex.reset_metrics()
        perm = torch.arange(data.n, device=ex.device)
        ex.train_step(data, perm, 0, data.n)
        loss, acc, _ = ex.read_metrics()
        return [loss, acc] if self.metrics else loss

    def test_on_batch(self, x, y):
        return self.evaluate(x, y, batch_size=len(x), verbose=0)

    # ------------------------------------------------------------------ summary
    def summary(self, line_length=None, positions=None, print_fn=None):
        print_fn = print_fn or print
        line_length = line_length or 65
        positions = positions or [0.45, 0.85, 1.0]
        if positions[-1] <= 1:
            positions = [int(line_length * p) for p in positions]

        def row(fields):
            line = ""
            for i, f in enumerate(fields):
                if i > 0:
                    line = line[:-1] + " "
                line += str(f)
                line = line[:positions[i]]
                line += " " * (positions[i] - len(line))
            print_fn(line)

        print_fn("_" * line_length)
        row(["Layer (type)", "Output Shape", "Param #"])
        print_fn("=" * line_length)
        shown = self._summary_layers()
        for i, layer in enumerate(shown):
            row(["%s (%s)" % (layer.name, type(layer).__name__), str(layer.output_shape),
                 layer.count_params()])
            print_fn("=" * line_length if i == len(shown) - 1 else "_" * line_length)
        total = self.count_params()
        trainable = sum(l.count_params() for l in self._chain if l.trainable)
        print_fn("Total params: {:,}".format(total))
        print_fn("Trainable params: {:,}".format(trainable))
        print_fn("Non-trainable params: {:,}".format(total - trainable))
        print_fn("_" * line_length)

    def _summary_layers(self):
        return self._chain

    # ------------------------------------------------------------------ serialisation
    def get_config(self):
        layers = []
        names = [l.name for l in self._chain]
        for i, l in enumerate(self._chain):
            inbound = [] if i == 0 else [[[names[i - 1], 0, 0, {}]]]
            layers.append({"name": l.name, "class_name": type(l).__name__, "config": l.get_config(),
                           "inbound_nodes": inbound})
        return {"name": self.name, "layers": layers,
                "input_layers": [[names[0], 0, 0]], "output_layers": [[names[-1], 0, 0]]}

    def to_json(self, **kw):
        import json
        return json.dumps({"class_name": type(self).__name__, "config": self.get_config(),
                           "keras_version": "2.2.4", "backend": "tensorflow"}, **kw)

    def save(self, filepath, overwrite=True, include_optimizer=True):
        from ..io.keras_h5 import save_model
        save_model(self, filepath, overwrite=overwrite, include_optimizer=include_optimizer)

    def save_weights(self, filepath, overwrite=True):
        from ..io.keras_h5 import save_weights
        save_weights(self, filepath)

    def load_weights(self, filepath, by_name=False):
        from ..io.keras_h5 import load_weights
        load_weights(self, filepath)


class Sequential(Model):
    def __init__(self, layers=None, name=None, device=None):
        super().__init__(name=name or "sequential_%d" % _seq_counter(), device=device)
        for l in layers or []:
            self.add(l)

    def add(self, layer: Layer):
        if not self._chain:
            if isinstance(layer, InputLayer):
                self._chain = [layer]
                return
            if layer.batch_input_shape is None:
                raise ValueError("The first layer in a Sequential model must get an "
                                 "`input_shape` argument.")
            inp = InputLayer(batch_input_shape=layer.batch_input_shape,
                             name=layer.name + "_input")
            self._chain = [inp]
        prev = self._chain[-1]
        layer.build(prev.output_shape_)
        self._chain.append(layer)
        self._build_store()
        self._compiled = False
        self._executor = None

    def pop(self):
        self._chain.pop()
        if len(self._chain) > 1:
            self._build_store()
        self._executor = None

    @property
    def layers(self):
        return [l for l in self._chain if not isinstance(l, InputLayer)]

    def _summary_layers(self):
        return self.layers

    def get_config(self):
        # Keras 2.2.4 form ({"name", "layers"}); 2.2.0's bare list is accepted on load
        return {"name": self.name,
                "layers": [{"class_name": type(l).__name__, "config": l.get_config()} for l in self.layers]}


_SEQ = [0]


def _seq_counter():
    _SEQ[0] += 1
    return _SEQ[0]
