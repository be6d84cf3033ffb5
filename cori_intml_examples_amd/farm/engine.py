"""Farm engine: one process per MI355X (``ipengine`` analogue, ``startCluster.sh:18``).

The controller starts engine ``i`` with ``HIP_VISIBLE_DEVICES=<gpu i>`` and the DP rank
environment (``RANK=i``, ``WORLD_SIZE=n``, ``LOCAL_RANK=0`` since one GPU is visible,
``MASTER_ADDR=127.0.0.1``), so ``hvd.init()`` inside ``%%px`` cells makes the engines the
ranks of one data-parallel job, exactly like the reference's Horovod-over-engines
workflow (``DistTrain_mnist.ipynb:148``) -- but with engine id == rank == GPU index
(the reference's engine ids and ranks differ, ``DistTrain_mnist.ipynb:133``).

Task kinds: ``apply`` (cloudpickled f, args, kwargs), ``execute`` (code in the engine
namespace), ``push`` (dict into the namespace), ``pull`` (``eval`` of names/expressions in
the namespace, as IPyParallel's ``_pull`` does -- ``c[0].get('history.epoch')`` at
``DistTrain_rpv.ipynb:310`` relies on it).

Running tasks stream stdout/stderr to the controller as they are written, can publish
live data (``publish_data``, ``mlextras.py:21-33``) and are cancellable: an ``interrupt``
sets the cooperative stop flag (``should_stop()``, checked by ``FarmStopCallback`` at
batch ends) and raises ``KeyboardInterrupt`` in the task; the controller hard-kills the
engine if the task does not end within its grace period.
"""
from __future__ import annotations

import _thread
import argparse
import io
import os
import queue
import sys
import threading
import time
import traceback
from multiprocessing.connection import Client as _Conn
from typing import Any, Dict, Optional

from . import protocol as P

_ENGINE: Optional["Engine"] = None


class _TaskStream(io.TextIOBase):
    def __init__(self, engine: "Engine", msg_id: str, name: str):
        self._e, self._id, self._name = engine, msg_id, name
        self._buf = []
        self._n = 0

    def writable(self):
        return True

    def write(self, s):
        if not s:
            return 0
        self._buf.append(s)
        self._n += len(s)
        if "\n" in s or self._n > 4096:
            self.flush()
        return len(s)

    def flush(self):
        if self._buf:
            text = "".join(self._buf)
            self._buf, self._n = [], 0
            self._e.send({"type": "stream", "msg_id": self._id, "name": self._name, "text": text})

    def isatty(self):
        return False


class Engine:
    def __init__(self, info: Dict[str, Any], engine_id: int):
        self.info = info
        self.engine_id = int(engine_id)
        self.conn = _Conn(info["address"], authkey=P.authkey(info))
        self._send_lock = threading.Lock()
        self.tasks: "queue.Queue" = queue.Queue()
        self.current: Optional[str] = None
        self.stop_flag = threading.Event()
        self.ns: Dict[str, Any] = {"__name__": "__engine__", "__builtins__": __builtins__}
        self.send({"type": "hello", "role": "engine", "engine_id": self.engine_id, "pid": os.getpid(),
                   "gpu": os.environ.get("HIP_VISIBLE_DEVICES")})

    def send(self, msg):
        with self._send_lock:
            self.conn.send(msg)

    # -- control reader ------------------------------------------------------------
    def _reader(self):
        while True:
            try:
                msg = self.conn.recv()
            except (EOFError, OSError):
                self.tasks.put(None)
                return
            t = msg.get("type")
            if t == "task":
                self.tasks.put(msg)
            elif t == "interrupt":
                if self.current is not None and msg.get("msg_id") == self.current:
                    self.stop_flag.set()
                    if not msg.get("cooperative_only"):
                        _thread.interrupt_main()
            elif t == "shutdown":
                self.tasks.put(None)
                return

    # -- task execution --------------------------------------------------------------
    def _run(self, msg):
        kind = msg["kind"]
        payload = P.loads(msg["payload"]) if msg.get("payload") is not None else None
        if kind == "apply":
            f, args, kwargs = payload
            return f(*args, **kwargs)
        if kind == "execute":
            exec(compile(payload, "<px>", "exec"), self.ns)
            return None
        if kind == "push":
            self.ns.update(payload)
            return None
        if kind == "pull":
            if isinstance(payload, (list, tuple)):
                return [eval(k, self.ns) for k in payload]
            return eval(payload, self.ns)
        raise ValueError("unknown task kind %r" % kind)

    # -- resource telemetry -------------------------------------------------------------
    def resource_stats(self) -> Dict[str, Any]:
        """This engine's GPU and memory use: HIP device (HIP_VISIBLE_DEVICES), HBM reserved /
        allocated by this process's caching allocator and the device total, host RSS.  Never
        initialises the GPU itself (a HIP call from this thread would)."""
        st: Dict[str, Any] = {"gpu": os.environ.get("HIP_VISIBLE_DEVICES"), "pid": os.getpid()}
        try:
            with open("/proc/self/statm") as f:
                st["rss_bytes"] = int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
        except (OSError, ValueError):
            pass
        torch = sys.modules.get("torch")
        try:
            if torch is not None and torch.cuda.is_initialized():
                dev = torch.cuda.current_device()
                st["hbm_reserved_bytes"] = int(torch.cuda.memory_reserved(dev))
                st["hbm_allocated_bytes"] = int(torch.cuda.memory_allocated(dev))
                st["hbm_peak_bytes"] = int(torch.cuda.max_memory_reserved(dev))
                st["hbm_total_bytes"] = int(torch.cuda.get_device_properties(dev).total_memory)
        except Exception:                # noqa: BLE001 - telemetry must never kill the engine
            pass
        return st

    def _telemetry(self, period: float):
        while True:
            time.sleep(period)
            try:
                self.send({"type": "stats", "stats": self.resource_stats()})
            except Exception:            # noqa: BLE001 - connection gone: the engine is exiting
                return

    def serve(self):
        global _ENGINE
        _ENGINE = self
        threading.Thread(target=self._reader, daemon=True, name="farm-engine-reader").start()
        period = float(os.environ.get("INTML_FARM_STATS_PERIOD", "2.0"))
        if period > 0:
            threading.Thread(target=self._telemetry, args=(period,), daemon=True, name="farm-engine-stats").start()
        while True:
            try:
                msg = self.tasks.get()
                if msg is None:
                    return
                self._execute(msg)
            except KeyboardInterrupt:     # a late interrupt that missed its task: ignore
                continue

    def _execute(self, msg):
        mid = msg["msg_id"]
        self.stop_flag.clear()
        out, err = _TaskStream(self, mid, "stdout"), _TaskStream(self, mid, "stderr")
        old = sys.stdout, sys.stderr
        self.current = mid
        self.send({"type": "started", "msg_id": mid, "t": P.now()})
        result = {"type": "result", "msg_id": mid}
        try:
            sys.stdout, sys.stderr = out, err
            try:
                value = self._run(msg)
                result.update(ok=True, value=P.dumps(value))
            except KeyboardInterrupt:
                result.update(ok=False, ename="TaskAborted", evalue="task interrupted",
                              traceback=traceback.format_exc())
            except BaseException as e:   # noqa: BLE001 - report everything to the client
                result.update(ok=False, ename=type(e).__name__, evalue=str(e), traceback=traceback.format_exc())
        finally:
            self.current = None
            try:
                out.flush()
                err.flush()
            finally:
                sys.stdout, sys.stderr = old
        result["t"] = P.now()
        try:
            self.send(result)
        except Exception:                # unpicklable value -> report as an error
            self.send({"type": "result", "msg_id": mid, "ok": False, "ename": "SerializationError",
                       "evalue": "task result could not be sent", "traceback": traceback.format_exc(),
                       "t": P.now()})


# ------------------------------------------------------------------------ engine-side API
def publish_data(data: Dict[str, Any]) -> None:
    """Publish a dict to the client: merged into ``AsyncResult.data`` of the running task
    (``ipyparallel.datapub.publish_data``, used by ``mlextras.py:21-33``).  Outside an
    engine task this is a no-op so the same training code runs standalone."""
    e = _ENGINE
    if e is None or e.current is None:
        return
    e.send({"type": "datapub", "msg_id": e.current, "data": P.dumps(dict(data))})


def engine_id() -> Optional[int]:
    return None if _ENGINE is None else _ENGINE.engine_id


_LOCAL_NS: Dict[str, Any] = {}


def engine_namespace() -> Dict[str, Any]:
    """The engine's persistent namespace (what ``push``/``pull``/``%%px`` see).  Functions
    shipped by value get fresh globals per task, so state that must survive across tasks
    on one engine (a resident dataset, a compiled model) is kept here.  Outside an engine
    this is a process-wide dict."""
    e = _ENGINE
    return _LOCAL_NS if e is None else e.ns


def should_stop() -> bool:
    """Cooperative cancellation flag of the running task (Stop button / ``AsyncResult.abort``)."""
    e = _ENGINE
    return bool(e is not None and e.stop_flag.is_set())


def main(argv=None):
    ap = argparse.ArgumentParser(description="intml farm engine")
    ap.add_argument("--cluster-id", default="default")
    ap.add_argument("--connection-file", default=None)
    ap.add_argument("--engine-id", type=int, required=True)
    a = ap.parse_args(argv)
    info = P.read_connection_file(a.cluster_id, a.connection_file)
    Engine(info, a.engine_id).serve()


if __name__ == "__main__":
    main()
