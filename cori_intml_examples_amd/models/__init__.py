"""Keras-shaped model API: layers, Sequential/Model, fused stage plan, executors."""
from .layers import Conv2D, Dense, Dropout, Flatten, Input, InputLayer, KTensor, Layer, MaxPooling2D, reset_names
from .model import Model, Sequential

__all__ = ["Layer", "InputLayer", "Input", "Conv2D", "MaxPooling2D", "Dropout", "Flatten", "Dense",
           "KTensor", "Model", "Sequential", "reset_names", "load_model"]


def load_model(filepath, custom_objects=None, compile=True):
    from ..io.keras_h5 import load_model as _lm
    return _lm(filepath, compile=compile)
