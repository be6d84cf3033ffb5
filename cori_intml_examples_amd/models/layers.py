"""Keras-2.2-shaped layer objects (symbolic only: no math lives here).

A layer records its configuration, its weight specs (Keras order and layout) and
its output shape.  Execution is done by the fused stage plan (``plan.py``) on
either the HIP backend (gfx950 kernels) or the CPU reference backend.

API parity targets: ``mnist.py:44-59`` (Sequential + Conv2D/MaxPooling2D/Dropout/
Flatten/Dense) and ``rpv.py:38-72`` (functional ``Input`` -> layers -> ``Model``).
Auto-naming reproduces Keras' per-class session counters (``conv2d_1``,
``max_pooling2d_1``, ... as printed at ``DistTrain_mnist.ipynb:266-283``).
"""
from __future__ import annotations

import re
from collections import defaultdict
from typing import Dict, List, Optional, Sequence, Tuple

from ..ops.reference import conv_out_size

_name_counters: Dict[str, int] = defaultdict(int)


def _snake(cls_name: str) -> str:
    # keras.engine.base_layer._to_snake_case
    s = re.sub(r"(.)([A-Z][a-z0-9]+)", r"\1_\2", cls_name)
    return re.sub(r"([a-z])([A-Z])", r"\1_\2", s).lower()


def unique_name(prefix: str) -> str:
    _name_counters[prefix] += 1
    return "%s_%d" % (prefix, _name_counters[prefix])


def reset_names() -> None:
    """Equivalent of ``keras.backend.clear_session()`` for layer auto-naming."""
    _name_counters.clear()


def _pair(v) -> Tuple[int, int]:
    if isinstance(v, (tuple, list)):
        assert len(v) == 2
        return int(v[0]), int(v[1])
    return int(v), int(v)


class KTensor:
    """Symbolic tensor of the functional API (shape excludes the batch axis)."""

    def __init__(self, shape: Tuple[int, ...], layer: "Layer", inbound: Optional["KTensor"]):
        self.shape = tuple(shape)
        self._keras_shape = (None,) + self.shape
        self.layer = layer
        self.inbound = inbound

    def __repr__(self):
        return "<KTensor shape=%s from %s>" % ((None,) + self.shape, self.layer.name)


class Layer:
    activation_names = (None, "linear", "relu", "softmax", "sigmoid")

    def __init__(self, name: Optional[str] = None, input_shape=None, trainable: bool = True, **kw):
        self.name = name or unique_name(_snake(type(self).__name__))
        self.trainable = trainable
        self.batch_input_shape = (None,) + tuple(input_shape) if input_shape is not None else None
        self.input_shape: Optional[Tuple[int, ...]] = None   # without batch axis
        self.output_shape_: Optional[Tuple[int, ...]] = None
        self.built = False
        self._weights: Dict[str, object] = {}   # filled by the param store (tensor views)
        self._inbound: Optional[KTensor] = None
        self.model = None

    # -- shapes ---------------------------------------------------------------------------
    def build(self, input_shape: Tuple[int, ...]) -> None:
        self.input_shape = tuple(input_shape)
        self.output_shape_ = tuple(self.compute_output_shape(self.input_shape))
        self.built = True

    def compute_output_shape(self, input_shape):
        return input_shape

    @property
    def output_shape(self):
        return (None,) + tuple(self.output_shape_) if self.output_shape_ is not None else None

    # -- weights --------------------------------------------------------------------------
    def weight_specs(self) -> List[Tuple[str, Tuple[int, ...], str]]:
        """[(short_name, shape, initializer)] in Keras order."""
        return []

    def count_params(self) -> int:
        n = 0
        for _, shape, _ in self.weight_specs():
            c = 1
            for s in shape:
                c *= s
            n += c
        return n

    @property
    def weights(self):
        return [self._weights[n] for n, _, _ in self.weight_specs()] if self._weights else []

    def get_weights(self):
        return [w.detach().cpu().numpy().copy() for w in self.weights]

    def set_weights(self, values) -> None:
        import torch
        specs = self.weight_specs()
        if len(values) != len(specs):
            raise ValueError("layer %s expects %d weights, got %d" % (self.name, len(specs), len(values)))
        for (n, shape, _), v in zip(specs, values):
            t = torch.as_tensor(v, dtype=torch.float32)
            if tuple(t.shape) != tuple(shape):
                raise ValueError("weight %s/%s shape %s != %s" % (self.name, n, tuple(t.shape), shape))
            self._weights[n].copy_(t.to(self._weights[n].device))
        if self.model is not None:
            self.model._weights_changed()

    # -- functional API -------------------------------------------------------------------
    def __call__(self, x: KTensor) -> KTensor:
        if not isinstance(x, KTensor):
            raise TypeError("layers are called on symbolic tensors from Input()")
        if self._inbound is not None:
            raise ValueError("layer %s is already connected (shared layers unsupported)" % self.name)
        self.build(x.shape)
        self._inbound = x
        return KTensor(self.output_shape_, self, x)

    def get_config(self) -> dict:
        cfg = {"name": self.name, "trainable": self.trainable}
        if self.batch_input_shape is not None:
            cfg["batch_input_shape"] = list(self.batch_input_shape)
            cfg["dtype"] = "float32"
        return cfg

    @classmethod
    def from_config(cls, cfg: dict) -> "Layer":
        cfg = dict(cfg)
        bis = cfg.pop("batch_input_shape", None)
        cfg.pop("dtype", None)
        if bis is not None:
            cfg["input_shape"] = tuple(bis[1:])
        return cls(**cfg)


class InputLayer(Layer):
    def __init__(self, input_shape=None, batch_input_shape=None, name=None, dtype="float32", **kw):
        if batch_input_shape is not None:
            input_shape = tuple(batch_input_shape[1:])
        super().__init__(name=name or unique_name("input"), input_shape=input_shape)
        self.build(tuple(input_shape))

    def get_config(self):
        return {"batch_input_shape": list(self.batch_input_shape), "dtype": "float32",
                "sparse": False, "name": self.name}

    @classmethod
    def from_config(cls, cfg):
        return cls(batch_input_shape=cfg["batch_input_shape"], name=cfg.get("name"))


def Input(shape=None, batch_shape=None, name=None, dtype="float32") -> KTensor:
    if shape is None and batch_shape is not None:
        shape = tuple(batch_shape[1:])
    layer = InputLayer(input_shape=tuple(shape), name=name)
    return KTensor(tuple(shape), layer, None)


def _check_act(act):
    if callable(act):
        act = getattr(act, "__name__", None)
    if act not in Layer.activation_names:
        raise ValueError("unsupported activation %r (supported: %s)" % (act, Layer.activation_names))
    return None if act == "linear" else act


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", data_format=None,
                 dilation_rate=(1, 1), activation=None, use_bias=True,
                 kernel_initializer="glorot_uniform", bias_initializer="zeros", **kw):
        super().__init__(**kw)
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        if self.strides[0] != self.strides[1]:
            raise NotImplementedError("anisotropic strides")
        if _pair(dilation_rate) != (1, 1):
            raise NotImplementedError("dilated convolutions")
        if data_format not in (None, "channels_last"):
            raise NotImplementedError("only channels_last (reference forces it, mnist.py:30)")
        padding = padding.lower()
        if padding not in ("valid", "same"):
            raise ValueError(padding)
        self.padding = padding
        self.activation = _check_act(activation)
        if self.activation in ("softmax",):
            raise NotImplementedError("softmax on a conv output")
        self.use_bias = bool(use_bias)
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer

    def compute_output_shape(self, s):
        if len(s) != 3:
            raise ValueError("Conv2D expects (H, W, C) inputs, got %s" % (s,))
        kh, kw = self.kernel_size
        st = self.strides[0]
        return (conv_out_size(s[0], kh, st, self.padding), conv_out_size(s[1], kw, st, self.padding),
                self.filters)

    def weight_specs(self):
        kh, kw = self.kernel_size
        cin = self.input_shape[-1]
        specs = [("kernel", (kh, kw, cin, self.filters), self.kernel_initializer)]
        if self.use_bias:
            specs.append(("bias", (self.filters,), self.bias_initializer))
        return specs

    def get_config(self):
        cfg = super().get_config()
        cfg.update({"filters": self.filters, "kernel_size": list(self.kernel_size),
                    "strides": list(self.strides), "padding": self.padding,
                    "data_format": "channels_last", "dilation_rate": [1, 1],
                    "activation": self.activation or "linear", "use_bias": self.use_bias,
                    "kernel_initializer": {"class_name": "VarianceScaling", "config": {
                        "scale": 1.0, "mode": "fan_avg", "distribution": "uniform", "seed": None}},
                    "bias_initializer": {"class_name": "Zeros", "config": {}},
                    "kernel_regularizer": None, "bias_regularizer": None,
                    "activity_regularizer": None, "kernel_constraint": None, "bias_constraint": None})
        return cfg

    @classmethod
    def from_config(cls, cfg):
        cfg = {k: v for k, v in cfg.items() if k in (
            "name", "trainable", "filters", "kernel_size", "strides", "padding", "activation",
            "use_bias", "batch_input_shape")}
        return super().from_config(cfg)


class MaxPooling2D(Layer):
    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", data_format=None, **kw):
        super().__init__(**kw)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        self.padding = padding
        if self.pool_size != (2, 2) or self.strides != (2, 2) or padding != "valid":
            raise NotImplementedError("only 2x2/2 'valid' max-pooling is implemented "
                                      "(the only form the reference uses)")

    def compute_output_shape(self, s):
        return (s[0] // 2, s[1] // 2, s[2])

    def get_config(self):
        cfg = super().get_config()
        cfg.update({"pool_size": list(self.pool_size), "padding": self.padding,
                    "strides": list(self.strides), "data_format": "channels_last"})
        return cfg

    @classmethod
    def from_config(cls, cfg):
        return cls(name=cfg.get("name"), pool_size=cfg.get("pool_size", (2, 2)),
                   strides=cfg.get("strides"), padding=cfg.get("padding", "valid"))


class Dropout(Layer):
    def __init__(self, rate, noise_shape=None, seed=None, **kw):
        super().__init__(**kw)
        self.rate = float(rate)
        if not 0.0 <= self.rate < 1.0:
            raise ValueError("dropout rate must be in [0, 1)")
        if noise_shape is not None:
            raise NotImplementedError("noise_shape")
        self.seed = seed

    def get_config(self):
        cfg = super().get_config()
        cfg.update({"rate": self.rate, "noise_shape": None, "seed": self.seed})
        return cfg

    @classmethod
    def from_config(cls, cfg):
        return cls(cfg["rate"], name=cfg.get("name"))


class Flatten(Layer):
    def __init__(self, data_format=None, **kw):
        super().__init__(**kw)

    def compute_output_shape(self, s):
        n = 1
        for v in s:
            n *= v
        return (n,)

    def get_config(self):
        cfg = super().get_config()
        cfg["data_format"] = "channels_last"
        return cfg

    @classmethod
    def from_config(cls, cfg):
        return cls(name=cfg.get("name"))


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", **kw):
        super().__init__(**kw)
        self.units = int(units)
        self.activation = _check_act(activation)
        self.use_bias = bool(use_bias)
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer

    def compute_output_shape(self, s):
        if len(s) != 1:
            raise ValueError("Dense expects flat inputs (add Flatten()), got %s" % (s,))
        return (self.units,)

    def weight_specs(self):
        specs = [("kernel", (self.input_shape[0], self.units), self.kernel_initializer)]
        if self.use_bias:
            specs.append(("bias", (self.units,), self.bias_initializer))
        return specs

    def get_config(self):
        cfg = super().get_config()
        cfg.update({"units": self.units, "activation": self.activation or "linear",
                    "use_bias": self.use_bias,
                    "kernel_initializer": {"class_name": "VarianceScaling", "config": {
                        "scale": 1.0, "mode": "fan_avg", "distribution": "uniform", "seed": None}},
                    "bias_initializer": {"class_name": "Zeros", "config": {}},
                    "kernel_regularizer": None, "bias_regularizer": None,
                    "activity_regularizer": None, "kernel_constraint": None, "bias_constraint": None})
        return cfg

    @classmethod
    def from_config(cls, cfg):
        cfg = {k: v for k, v in cfg.items() if k in (
            "name", "trainable", "units", "activation", "use_bias", "batch_input_shape")}
        return super().from_config(cfg)


LAYER_CLASSES = {c.__name__: c for c in (InputLayer, Conv2D, MaxPooling2D, Dropout, Flatten, Dense)}
