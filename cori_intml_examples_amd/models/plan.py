"""Fused stage plan: groups a Keras layer chain into the kernels that execute it.

The reference runs every Keras layer as separate TF ops.  Here a
model is compiled into *stages*, each of which maps onto one fused HIP kernel
family on gfx950:

  ConvStage   Conv2D(+ReLU) [+MaxPool 2x2] [+Dropout]   -> conv_mm (fwd epilogue)
  DenseStage  Dense(+ReLU) [+Dropout]                   -> dense split-K + epilogue
  HeadStage   final Dense + softmax/sigmoid + loss      -> head_fused (fwd+loss+bwd)

The plan is backend-agnostic; executors (``executor_ref`` / ``executor_hip``)
interpret it.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from .layers import Conv2D, Dense, Dropout, Flatten, InputLayer, Layer, MaxPooling2D
from ..ops.reference import conv_pads


@dataclass
class ConvStage:
    conv: Conv2D
    in_shape: Tuple[int, int, int]          # H, W, Cin
    conv_shape: Tuple[int, int, int]        # Ho, Wo, Cout (pre-pool)
    out_shape: Tuple[int, int, int]         # post-pool shape
    relu: bool
    pool: Optional[MaxPooling2D] = None
    dropout: Optional[Dropout] = None
    stream: int = 0                         # RNG stream id of the dropout

    @property
    def rate(self) -> float:
        return self.dropout.rate if self.dropout is not None else 0.0

    @property
    def stride(self) -> int:
        return self.conv.strides[0]

    @property
    def pads(self):
        H, W, _ = self.in_shape
        kh, kw = self.conv.kernel_size
        return conv_pads(H, W, kh, kw, self.stride, self.conv.padding)


@dataclass
class DenseStage:
    dense: Dense
    K: int
    N: int
    relu: bool
    dropout: Optional[Dropout] = None
    stream: int = 0
    flat_from: Optional[Tuple[int, int, int]] = None   # (H,W,C) if the input comes from a Flatten

    @property
    def rate(self) -> float:
        return self.dropout.rate if self.dropout is not None else 0.0


@dataclass
class HeadStage:
    dense: Dense
    K: int
    N: int
    activation: Optional[str]     # 'softmax' | 'sigmoid' | None
    loss: str                     # canonical loss name
    flat_from: Optional[Tuple[int, int, int]] = None


@dataclass
class Plan:
    input_shape: Tuple[int, ...]
    convs: List[ConvStage] = field(default_factory=list)
    denses: List[DenseStage] = field(default_factory=list)
    head: Optional[HeadStage] = None

    @property
    def stages(self):
        return list(self.convs) + list(self.denses) + ([self.head] if self.head else [])


def canonical_loss(loss) -> str:
    name = loss if isinstance(loss, str) else getattr(loss, "__name__", str(loss))
    aliases = {"categorical_crossentropy": "categorical_crossentropy",
               "binary_crossentropy": "binary_crossentropy",
               "mse": "mse", "mean_squared_error": "mse",
               "sparse_categorical_crossentropy": "sparse_categorical_crossentropy"}
    if name not in aliases:
        raise NotImplementedError("loss %r is not implemented" % (name,))
    return aliases[name]


def build_plan(layers: List[Layer], loss) -> Plan:
    """``layers`` is the linear chain starting with an InputLayer."""
    if not layers or not isinstance(layers[0], InputLayer):
        raise ValueError("model must start with an input layer")
    loss = canonical_loss(loss)
    plan = Plan(input_shape=tuple(layers[0].output_shape_))
    cur_conv: Optional[ConvStage] = None
    cur_dense: Optional[DenseStage] = None
    flat_from = None
    body = layers[1:]
    stream = 0
    for i, layer in enumerate(body):
        last = i == len(body) - 1
        if isinstance(layer, Conv2D):
            if plan.denses or flat_from is not None:
                raise NotImplementedError("Conv2D after Flatten/Dense")
            relu = layer.activation == "relu"
            if layer.activation not in (None, "relu"):
                raise NotImplementedError("conv activation %s" % layer.activation)
            cur_conv = ConvStage(conv=layer, in_shape=tuple(layer.input_shape),
                                 conv_shape=tuple(layer.output_shape_),
                                 out_shape=tuple(layer.output_shape_), relu=relu)
            plan.convs.append(cur_conv)
            cur_dense = None
        elif isinstance(layer, MaxPooling2D):
            if cur_conv is None or cur_conv.pool is not None or cur_conv.dropout is not None:
                raise NotImplementedError("MaxPooling2D must directly follow a Conv2D")
            cur_conv.pool = layer
            cur_conv.out_shape = tuple(layer.output_shape_)
        elif isinstance(layer, Dropout):
            stream += 1
            tgt = cur_dense if cur_dense is not None else cur_conv
            if tgt is None:
                raise NotImplementedError("Dropout directly on the model input")
            if tgt.dropout is not None:
                raise NotImplementedError("two consecutive Dropout layers")
            tgt.dropout = layer
            tgt.stream = stream
        elif isinstance(layer, Flatten):
            if flat_from is not None or plan.denses:
                raise NotImplementedError("Flatten after Dense")
            flat_from = tuple(layer.input_shape)
        elif isinstance(layer, Dense):
            if len(layer.input_shape) != 1:
                raise ValueError("Dense on non-flat input")
            ff = flat_from if not plan.denses else None
            if last:
                act = layer.activation
                if act not in (None, "softmax", "sigmoid"):
                    raise NotImplementedError("output activation %s" % act)
                plan.head = HeadStage(dense=layer, K=layer.input_shape[0], N=layer.units,
                                      activation=act, loss=loss, flat_from=ff)
            else:
                if layer.activation not in (None, "relu"):
                    raise NotImplementedError("hidden Dense activation %s" % layer.activation)
                cur_dense = DenseStage(dense=layer, K=layer.input_shape[0], N=layer.units,
                                       relu=layer.activation == "relu", flat_from=ff)
                plan.denses.append(cur_dense)
            cur_conv = None
        else:
            raise NotImplementedError("layer type %s" % type(layer).__name__)
    if plan.head is None:
        raise NotImplementedError("the model must end with a Dense layer")
    if plan.head.activation == "softmax" and loss not in ("categorical_crossentropy",
                                                          "sparse_categorical_crossentropy"):
        raise NotImplementedError("softmax output with loss %s" % loss)
    if plan.head.activation == "sigmoid" and loss != "binary_crossentropy":
        raise NotImplementedError("sigmoid output with loss %s" % loss)
    return plan
