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
import time
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

    # ------------------------------------------------------------------ admission
    def self_test(self, timeout_s: float = 60.0) -> Optional[str]:
        """Closed-form numeric all-reduce, eager AND captured into a HIP graph (the way the
        training step issues it): rank r contributes (r + 1) * (i % 13 + 1), so every element
        of the sum is the exact integer size (size + 1) / 2 * (i % 13 + 1) in fp32.  Bounded
        in time: a collective that does not complete within ``timeout_s`` aborts the
        communicator.  Returns None on success, else what went wrong (for the init vote)."""
        dev = self.device
        n = 4099                                   # odd: not a multiple of any RCCL chunking
        base = (torch.arange(n, device=dev, dtype=torch.float32) % 13) + 1
        want = base * (self.size * (self.size + 1) / 2)
        mine = base * (self.rank + 1)

        def wait(what: str) -> Optional[str]:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            deadline = time.monotonic() + timeout_s
            while not ev.query():
                if time.monotonic() > deadline:
                    self.abort("self-test %s did not complete within %.0f s" % (what, timeout_s))
                    return "%s all-reduce timed out after %.0f s" % (what, timeout_s)
                time.sleep(1e-3)
            return None

        try:
            with torch.cuda.device(dev):
                t = mine.clone()
                self.all_reduce(t)
                err = wait("eager")
                if err:
                    return err
                if not torch.equal(t, want):
                    return "eager all-reduce wrong: max |err| %.3g" % float((t - want).abs().max())
                t2 = torch.zeros_like(mine)
                s = torch.cuda.Stream(device=dev)
                s.wait_stream(torch.cuda.current_stream(dev))
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    self.all_reduce(t2, stream=s)
                t2.copy_(mine)
                g.replay()
                err = wait("captured")
                if err:
                    return err
                if not torch.equal(t2, want):
                    return "captured all-reduce wrong: max |err| %.3g" % float((t2 - want).abs().max())
                del g
        except Exception as e:   # noqa: BLE001 -- reported through the vote
            return "%s: %s" % (type(e).__name__, e)
        return None


def establish(rank: int, size: int, device: torch.device, timeout_s: float = 600.0,
              init_timeout_s: Optional[float] = None, factory=None):
    """Bring up the RCCL data plane for a job of ``size`` ranks, with the SAME outcome on every
    rank: returns ``(comm, None)`` or ``(None, [(rank, why), ...])``, in which case every rank
    runs the RCCL-free xGMI plane.  Each phase ends in a collective step of the gloo control
    plane, so an asymmetric failure -- one rank's only -- still reaches every rank:

      1. rank 0 creates the unique id (or reports why it could not) and broadcasts THAT, so a
         rank-0 failure does not leave the others inside a broadcast that never matches;
      2. every rank builds its communicator in a worker thread with a deadline
         (``INTML_RCCL_INIT_TIMEOUT``, default 120 s): a rank that never joins (it failed
         before ``ncclCommInitRank``) leaves its peers blocked inside RCCL, but their main
         threads give up waiting and go on to the vote (the blocked thread goes to a reaper
         that aborts + closes the communicator if it still comes up: ``_reap_late_init``);
      3. the numeric self-test (``NativeComm.self_test``: eager + graph-captured, closed-form);
      4. ONE all_gather of every rank's verdict; any failure anywhere -> every rank aborts its
         communicator and falls back.

    ``factory(rank, size, device, timeout_s, uid)`` builds a communicator (tests inject
    failing ones)."""
    import threading

    import torch.distributed as tdist
    factory = factory or (lambda r, n, d, t, u: NativeComm(r, n, d, t, uid=u))
    if init_timeout_s is None:
        init_timeout_s = float(os.environ.get("INTML_RCCL_INIT_TIMEOUT", 120))
    why = None
    # phase 1: the unique id, or rank 0's reason for not having one
    box = [None]
    if rank == 0:
        try:
            box = [("ok", _module().unique_id())]
        except Exception as e:   # noqa: BLE001
            box = [("err", "unique id: %s: %s" % (type(e).__name__, e))]
    if size > 1:
        tdist.broadcast_object_list(box, src=0)
    kind, val = box[0]
    comm = None
    if kind != "ok":
        why = val if rank == 0 else None
    else:
        # phase 2: communicator construction with a deadline
        res = {}

        def work():
            try:
                if device.type == "cuda":
                    torch.cuda.set_device(device)
                res["comm"] = factory(rank, size, device, timeout_s, val)
            except BaseException as e:   # noqa: BLE001
                res["err"] = "%s: %s" % (type(e).__name__, e)

        th = threading.Thread(target=work, name="rccl-init", daemon=True)
        th.start()
        th.join(init_timeout_s)
        if th.is_alive():
            why = "communicator not up within %.0f s (a peer never joined)" % init_timeout_s
            _reap_late_init(th, res)
        elif "err" in res:
            why = res["err"]
        else:
            comm = res["comm"]
            # phase 3: numeric self-test, eager and captured
            why = comm.self_test(min(timeout_s, 60.0))
    # phase 4: one vote
    votes = [why]
    if size > 1:
        votes = [None] * size
        tdist.all_gather_object(votes, why)
    bad = [(i, v) for i, v in enumerate(votes) if v]
    if bad:
        if comm is not None:
            try:
                comm.abort("data-plane vote failed: %s" % bad)
            except Exception:   # noqa: BLE001
                pass
            comm.close()
        return None, bad
    return comm, None


# communicator-init threads abandoned at their deadline, and what became of them: "pending",
# "failed: ..." or "closed" (a late communicator is aborted + closed by the reaper, never used)
abandoned_inits: list = []


def _reap_late_init(th, res: dict) -> None:
    """An init thread that missed its deadline may still complete inside ncclCommInitRank
    later (its peers joined late).  By then the job has voted onto the RCCL-free plane, so a
    late communicator must not live on with its watchdog: a daemon reaper joins the thread and
    aborts + closes whatever it produced.  The outcome is recorded in ``abandoned_inits``."""
    import threading
    rec = {"thread": th.name, "state": "pending"}
    abandoned_inits.append(rec)

    def reap():
        th.join()
        c = res.get("comm")
        if c is None:
            rec["state"] = "failed: %s" % res.get("err", "no communicator")
            return
        try:
            c.abort("communicator came up after the init deadline; the job runs without RCCL")
        except Exception:   # noqa: BLE001
            pass
        try:
            c.close()
        finally:
            rec["state"] = "closed"

    threading.Thread(target=reap, name="rccl-init-reaper", daemon=True).start()


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
