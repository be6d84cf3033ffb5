"""Python side of the native RCCL data-plane engine (``csrc/comm/engine.cpp``).

Control plane vs data plane:
  * control plane = a ``gloo`` torch.distributed group over TCP (127.0.0.1): rendezvous,
    the RCCL unique-id exchange, barriers, object gathers, host-scalar metric averages;
  * data plane = ONE RCCL communicator per process driven from C++: gradient buckets,
    state broadcast, device-tensor all-reduce.  Every call enqueues on a HIP stream and
    returns, so the executor captures the gradient all-reduces INTO the step's HIP graph.

Reference call sites served: ``hvd.init`` (train_rpv.py:37), ``DistributedOptimizer``
all-reduce (rpv.py:65), ``BroadcastGlobalVariablesCallback`` (rpv.py:85),
``MetricAverageCallback`` (rpv.py:87).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3,
           torch.int32: 4, torch.int64: 5, torch.uint8: 6}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


class _stdout_to_stderr:
    """Route fd 1 to fd 2 for the duration (library banners must not mix with a program's
    machine-readable stdout, e.g. bench.py's single JSON line)."""

    def __enter__(self):
        import ctypes
        import sys
        self._libc = ctypes.CDLL(None)
        sys.stdout.flush()
        self._libc.fflush(None)
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        import sys
        sys.stdout.flush()
        self._libc.fflush(None)
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


def _module():
    from .. import _comm          # built in-tree by _build.build_comm
    return _comm


def available() -> bool:
    try:
        _module()
        return True
    except ImportError:
        return False


class NativeComm:
    """One RCCL communicator (rank ``rank`` of ``size``) on the current HIP device."""

    def __init__(self, rank: int, size: int, device: torch.device, timeout_s: float = 600.0,
                 uid: Optional[bytes] = None):
        import torch.distributed as tdist
        m = _module()
        self.rank, self.size, self.device = rank, size, device
        if uid is None:
            box = [m.unique_id() if rank == 0 else None]
            if size > 1:
                tdist.broadcast_object_list(box, src=0)    # over the gloo control plane
            uid = box[0]
        with _stdout_to_stderr():      # RCCL prints a version banner on stdout at init
            self._c = m.Comm(uid, size, rank, device.index if device.index is not None else 0)
            self.timeout_s = timeout_s
            if timeout_s and timeout_s > 0:
                self._c.start_watchdog(float(timeout_s))
            # one-time connection setup outside any graph capture (RCCL connects lazily on
            # the first collective, which must not happen inside a capture)
            t = torch.zeros(256, dtype=torch.float32, device=device)
            self.all_reduce(t)
            torch.cuda.current_stream(device).synchronize()

    @property
    def nranks(self) -> int:
        """Rank count as reported by the RCCL communicator (ncclCommCount)."""
        return self._c.comm_count()

    @property
    def comm_rank(self) -> int:
        return self._c.comm_rank()

    # ------------------------------------------------------------------ collectives
    @staticmethod
    def _stream(stream) -> int:
        if stream is None:
            return torch.cuda.current_stream().cuda_stream
        return stream if isinstance(stream, int) else stream.cuda_stream

    def all_reduce(self, t: torch.Tensor, op: str = "sum", stream=None, out: Optional[torch.Tensor] = None):
        """In-place (or into ``out``) all-reduce of a contiguous device tensor."""
        assert t.is_cuda and t.is_contiguous()
        dst = t if out is None else out
        self._c.all_reduce(t.data_ptr(), dst.data_ptr(), t.numel(), _DTYPES[t.dtype], _OPS[op], self._stream(stream))
        return dst

    def all_reduce_ptr(self, ptr: int, count: int, dtype=torch.float32, op: str = "sum", stream=None):
        self._c.all_reduce(ptr, ptr, count, _DTYPES[dtype], _OPS[op], self._stream(stream))

    def broadcast(self, t: torch.Tensor, root: int = 0, stream=None):
        assert t.is_cuda and t.is_contiguous()
        self._c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPES[t.dtype], root, self._stream(stream))
        return t

    def reduce_scatter(self, t: torch.Tensor, out: torch.Tensor, op: str = "sum", stream=None):
        assert t.numel() == out.numel() * self.size
        self._c.reduce_scatter(t.data_ptr(), out.data_ptr(), out.numel(), _DTYPES[t.dtype], _OPS[op],
                               self._stream(stream))
        return out

    def all_gather(self, t: torch.Tensor, out: torch.Tensor, stream=None):
        assert out.numel() == t.numel() * self.size
        self._c.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), _DTYPES[t.dtype], self._stream(stream))
        return out

    # ------------------------------------------------------------------ failure detection
    def mark(self, stream=None) -> None:
        """Step marker for the watchdog (call outside graph capture)."""
        self._c.mark(self._stream(stream))

    def check(self) -> None:
        self._c.check()

    @property
    def failed(self) -> bool:
        return self._c.failed

    @property
    def error(self) -> str:
        return self._c.error

    def abort(self, why: str = "aborted") -> None:
        self._c.abort(why)

    def close(self) -> None:
        if self._c is not None:
            self._c.stop_watchdog()
            self._c = None


def comm_mode(use_gpu: bool, backend: Optional[str], local_size: Optional[int] = None,
              n_devices: Optional[int] = None) -> str:
    """'native' (RCCL engine + gloo control plane), 'xgmi' (NO RCCL communicator: the fused
    xGMI all-reduce + optimizer kernel is the data plane, gloo the control plane) or 'torch'
    (torch.distributed only).

    ``INTML_COMM=torch`` forces the torch.distributed data plane and ``INTML_COMM=xgmi`` the
    RCCL-free one; an explicit ``INTML_DP_BACKEND``/``backend`` keeps the torch path.  With
    more ranks on this node than GPUs (ranks sharing a GPU: nested HPO x DP evaluations on
    one card, the one-GPU rehearsal of the 8-GPU step) RCCL refuses to build a communicator,
    so the native mode becomes 'xgmi': its protocol does not care whether a peer's inbox is
    on this GPU or another."""
    mode = os.environ.get("INTML_COMM", "native").lower()
    if not use_gpu or mode == "torch" or backend or os.environ.get("INTML_DP_BACKEND"):
        return "torch"
    if mode == "xgmi":
        return "xgmi"
    if local_size is not None and n_devices and local_size > n_devices:
        return "xgmi"
    if not available():
        raise RuntimeError("INTML_COMM=native but the _comm extension is not built "
                           "(python -m cori_intml_examples_amd._build); set INTML_COMM=torch to "
                           "use torch.distributed for the data plane")
    return "native"
