"""cori_intml_examples_amd — MI355X-native interactive distributed deep learning + HPO.

Capabilities of mlhenderson/cori-intml-examples re-designed for gfx950: Keras-shaped
CNN models whose layer stack runs on hand-written CDNA4 HIP kernels, Horovod-shaped
synchronous data parallelism over RCCL, an IPyParallel-shaped one-node task farm, and
random / genetic / grid hyper-parameter search with live monitoring widgets.
"""
__version__ = "0.1.0"

from . import models, optim, train, utils  # noqa: F401
from .models import (Conv2D, Dense, Dropout, Flatten, Input, MaxPooling2D, Model, Sequential,  # noqa: F401
                     load_model)
