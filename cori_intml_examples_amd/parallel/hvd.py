"""Drop-in for ``import horovod.keras as hvd`` (``train_rpv.py:10``, ``rpv.py:64,82``)."""
from . import callbacks
from .dist import (Compression, DataParallelDivergence, DistributedOptimizer, allgather, allreduce, barrier, broadcast,
                   broadcast_model_state, broadcast_object, init, is_initialized, local_rank,
                   local_size, rank, shutdown, size)


def broadcast_global_variables(root_rank=0, model=None):
    if model is not None:
        broadcast_model_state(model, root_rank)


__all__ = ["init", "shutdown", "rank", "size", "local_rank", "local_size", "allreduce",
           "allgather", "broadcast", "broadcast_object", "barrier", "DistributedOptimizer",
           "Compression", "callbacks", "broadcast_global_variables", "is_initialized",
           "DataParallelDivergence"]
