"""Data-parallel runtime (Horovod-shaped API over torch.distributed / RCCL).

``from cori_intml_examples_amd.parallel import hvd`` gives the drop-in module used as
``import horovod.keras as hvd`` in the reference (``train_rpv.py:10``).
"""
from . import callbacks, dist, state
from . import hvd

__all__ = ["dist", "state", "callbacks", "hvd"]
