"""Farm client: ``Client`` / ``DirectView`` / ``LoadBalancedView`` / ``AsyncResult``
with IPyParallel's call shapes (SURVEY.md §2.9 "Task-farm API"):

    c = Client(timeout=60, cluster_id='cori_%s' % job_id)      # DistTrain_mnist.ipynb:67-73
    c.ids; c[0].get('history.epoch'); c[:].get('history.history')   # DistTrain_rpv.ipynb:310-311
    lv = c.load_balanced_view()                                  # DistHPO_mnist.ipynb:240
    ar = lv.apply(build_and_train, **hp)                         # :249
    ar.ready(); ar.get(); ar.stdout; ar.stderr; ar.started; ar.completed; ar.data

A background receiver thread applies the controller's streamed events (started,
stdout/stderr chunks, ``publish_data`` dicts, results) to the AsyncResults, so progress
fields are live while the task runs (what the widget polls, ``hpo_widgets.py:254-323``).
"""
from __future__ import annotations

import threading
import time
from multiprocessing import AuthenticationError
from multiprocessing.connection import Client as _Conn
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Union

from . import protocol as P
from .protocol import EngineError, RemoteError, TaskAborted


class _TaskRecord:
    __slots__ = ("msg_id", "engine_id", "submitted", "started", "completed", "stdout", "stderr", "data",
                 "ok", "value", "error", "event", "callbacks", "status")

    def __init__(self, msg_id):
        self.msg_id = msg_id
        self.engine_id = None
        self.submitted = P.now()
        self.started = None
        self.completed = None
        self.stdout = ""
        self.stderr = ""
        self.data: Dict[str, Any] = {}
        self.ok = None
        self.value = None
        self.error: Optional[RemoteError] = None
        self.event = threading.Event()
        self.callbacks: List[Callable] = []
        self.status = "queued"


class AsyncResult:
    """Handle on one or more submitted tasks.  ``single`` results unwrap to a scalar."""

    def __init__(self, client: "Client", msg_ids: List[str], single: bool, mapper: Optional[Callable] = None):
        self._client = client
        self.msg_ids = list(msg_ids)
        self._single = single
        self._mapper = mapper

    # -- state ----------------------------------------------------------------------
    def _recs(self) -> List[_TaskRecord]:
        return [self._client._records[m] for m in self.msg_ids]

    def ready(self) -> bool:
        return all(r.event.is_set() for r in self._recs())

    done = ready

    def wait(self, timeout: float = -1) -> bool:
        deadline = None if timeout is None or timeout < 0 else time.time() + timeout
        for r in self._recs():
            left = None if deadline is None else max(0.0, deadline - time.time())
            if not r.event.wait(left):
                return False
        return True

    def successful(self) -> bool:
        if not self.ready():
            raise RuntimeError("task not finished")
        return all(r.ok for r in self._recs())

    def get(self, timeout: float = -1):
        if not self.wait(timeout):
            raise TimeoutError("Result not ready.")
        vals = []
        for r in self._recs():
            if not r.ok:
                raise r.error
            vals.append(r.value)
        if self._mapper is not None:
            return self._mapper(vals)
        return vals[0] if self._single else vals

    result = get

    def abort(self, grace: Optional[float] = None) -> None:
        """Cancel: queued tasks are dropped; running ones are interrupted (cooperative flag
        + KeyboardInterrupt) and their engine is killed and restarted after ``grace`` s."""
        self._client.abort(self.msg_ids, grace=grace)

    def add_done_callback(self, fn: Callable[["AsyncResult"], None]) -> None:
        pending = [r for r in self._recs() if not r.event.is_set()]
        if not pending:
            fn(self)
            return
        state = {"n": len(pending)}
        lock = threading.Lock()

        def one(_):
            with lock:
                state["n"] -= 1
                last = state["n"] == 0
            if last:
                fn(self)

        for r in pending:
            self._client._add_callback(r, one)

    # -- fields ----------------------------------------------------------------------
    def _field(self, name):
        vals = [getattr(r, name) for r in self._recs()]
        return vals[0] if self._single else vals

    @property
    def stdout(self):
        return self._field("stdout")

    @property
    def stderr(self):
        return self._field("stderr")

    @property
    def started(self):
        return self._field("started")

    @property
    def completed(self):
        return self._field("completed")

    @property
    def submitted(self):
        return self._field("submitted")

    @property
    def engine_id(self):
        return self._field("engine_id")

    @property
    def data(self):
        return self._field("data")

    @property
    def status(self):
        return self._field("status")

    @property
    def metadata(self):
        md = [{"msg_id": r.msg_id, "engine_id": r.engine_id, "submitted": r.submitted, "started": r.started,
               "completed": r.completed, "status": r.status, "stdout": r.stdout, "stderr": r.stderr,
               "data": r.data, "pyerr": r.error} for r in self._recs()]
        return md[0] if self._single else md

    @property
    def elapsed(self) -> float:
        recs = self._recs()
        end = max((r.completed or P.now()) for r in recs)
        return (end - min(r.submitted for r in recs)).total_seconds()

    @property
    def progress(self) -> int:
        return sum(1 for r in self._recs() if r.event.is_set())

    def __len__(self):
        return len(self.msg_ids)

    def __iter__(self):
        v = self.get()
        return iter(v if isinstance(v, list) else [v])

    def __repr__(self):
        st = "finished" if self.ready() else "pending"
        return "<AsyncResult: %s (%d task%s)>" % (st, len(self.msg_ids), "" if len(self.msg_ids) == 1 else "s")


class _View:
    block = False

    def __init__(self, client: "Client"):
        self.client = client

    def apply(self, f, *args, **kwargs):
        ar = self._submit_apply(f, args, kwargs)
        return ar.get() if self.block else ar

    def apply_async(self, f, *args, **kwargs):
        return self._submit_apply(f, args, kwargs)

    def apply_sync(self, f, *args, **kwargs):
        return self._submit_apply(f, args, kwargs).get()

    def map(self, f, *sequences, block=None):
        items = list(zip(*sequences))
        ids = [self.client._submit(self._target_for(i), "apply", (f, item, {})) for i, item in enumerate(items)]
        ar = AsyncResult(self.client, ids, single=False)
        return ar.get() if (self.block if block is None else block) else ar

    def map_sync(self, f, *sequences):
        return self.map(f, *sequences, block=True)

    def map_async(self, f, *sequences):
        return self.map(f, *sequences, block=False)

    def wait(self, jobs=None, timeout=-1):
        return self.client.wait(jobs, timeout)


class LoadBalancedView(_View):
    """Tasks go to whichever engine is idle first (``lv.apply``, ``DistHPO_mnist.ipynb:240-255``)."""

    def __init__(self, client, targets=None):
        super().__init__(client)
        self.targets = targets
        self._next = 0                 # round-robin position over an explicit target list

    def _target_for(self, i):
        if self.targets is None:
            return None
        t = self.targets if isinstance(self.targets, list) else [self.targets]
        return t[i % len(t)]

    def _submit_apply(self, f, args, kwargs):
        # no targets: the controller's shared queue (whichever engine is idle first); an
        # explicit target list: round-robin over it (the controller queues per engine)
        target = None
        if self.targets is not None:
            target = self._target_for(self._next)
            self._next += 1
        mid = self.client._submit(target, "apply", (f, tuple(args), dict(kwargs)))
        return AsyncResult(self.client, [mid], single=True)

    def __repr__(self):
        return "<LoadBalancedView None>"


class DirectView(_View):
    """SPMD view over explicit engines: ``c[:]``, ``c[0]`` (``%%px``, ``c[i].get``)."""

    def __init__(self, client, targets: Union[int, List[int]]):
        super().__init__(client)
        self._single = isinstance(targets, int)
        self.targets = [targets] if self._single else list(targets)

    def _target_for(self, i):
        return self.targets[i % len(self.targets)]

    def _fanout(self, kind, payload, block=None, mapper=None):
        ids = [self.client._submit(t, kind, payload) for t in self.targets]
        ar = AsyncResult(self.client, ids, single=self._single, mapper=mapper)
        return ar.get() if (self.block if block is None else block) else ar

    def _submit_apply(self, f, args, kwargs):
        ids = [self.client._submit(t, "apply", (f, tuple(args), dict(kwargs))) for t in self.targets]
        return AsyncResult(self.client, ids, single=self._single)

    def execute(self, code: str, block=None, silent=False):
        return self._fanout("execute", code, block)

    def run(self, filename: str, block=None):
        with open(filename) as f:
            return self.execute(f.read(), block)

    def push(self, ns: Dict[str, Any], block=None):
        return self._fanout("push", dict(ns), block)

    def pull(self, names, block=True):
        return self._fanout("pull", names, block)

    def get(self, name):
        return self.pull(name, block=True)

    def update(self, ns):
        return self.push(ns, block=True)

    def __getitem__(self, name):
        return self.get(name)

    def __setitem__(self, name, value):
        self.push({name: value}, block=True)

    def scatter(self, name: str, seq: Sequence, block=None):
        n = len(self.targets)
        chunks = [seq[i::n] for i in range(n)] if not hasattr(seq, "shape") else \
            [seq[(len(seq) * i) // n:(len(seq) * (i + 1)) // n] for i in range(n)]
        ids = [self.client._submit(t, "push", {name: chunks[i]}) for i, t in enumerate(self.targets)]
        ar = AsyncResult(self.client, ids, single=False)
        return ar.get() if (self.block if block is None else block) else ar

    def gather(self, name: str, block=True):
        import numpy as np
        parts = self.pull(name, block=True)
        parts = parts if isinstance(parts, list) else [parts]
        if parts and hasattr(parts[0], "shape"):
            return np.concatenate(parts)
        out = []
        for p in parts:
            out.extend(p)
        return out

    def abort(self, jobs=None):
        self.client.abort(jobs)

    def __len__(self):
        return len(self.targets)

    def __repr__(self):
        return "<DirectView %s>" % (self.targets[0] if self._single else self.targets)


class Client:
    """Connect to a running farm by ``cluster_id`` (``ipp.Client(timeout=60, cluster_id=…)``)."""

    def __init__(self, url_file: Optional[str] = None, profile: Optional[str] = None,
                 cluster_id: Optional[str] = None, timeout: float = 60, connection_info: Optional[dict] = None,
                 **kw):
        deadline = time.time() + float(timeout)
        info = connection_info
        while info is None:
            try:
                info = P.read_connection_file(cluster_id or "default", url_file)
            except (FileNotFoundError, ValueError):
                if time.time() > deadline:
                    raise TimeoutError("no farm cluster %r found (start one with startCluster / "
                                       "farm.start_cluster)" % (cluster_id or "default"))
                time.sleep(0.2)
        self.cluster_id = info["cluster_id"]
        self._conn = None
        while True:
            try:
                self._conn = _Conn(info["address"], authkey=P.authkey(info))
                break
            except (OSError, EOFError, AuthenticationError):
                # not listening yet, or a handshake cut short (controller busy / restarting):
                # transient until the deadline
                if time.time() > deadline:
                    raise TimeoutError("farm controller for %r is not accepting connections" % self.cluster_id)
                time.sleep(0.2)
        self._send_lock = threading.Lock()
        self._records: Dict[str, _TaskRecord] = {}
        self._rec_lock = threading.Lock()
        self._replies: Dict[str, dict] = {}
        self._reply_cv = threading.Condition()
        self._ids: List[int] = []
        self.info = {}
        self.engine_events: List[dict] = []
        self._closed = False
        rid = P.new_msg_id()
        self._conn.send({"type": "hello", "role": "client", "req_id": rid})
        hello = self._conn.recv()
        self._ids = hello.get("ids", [])
        self.info = hello.get("info", {})
        self._thread = threading.Thread(target=self._recv_loop, daemon=True, name="farm-client")
        self._thread.start()
        # wait for the engines to register (the reference's notebooks wait on len(c.ids))
        n = self.info.get("n_engines", 0)
        while len(self._ids) < n and time.time() < deadline:
            self._ids = self._request({"type": "ids"}).get("ids", [])
            if len(self._ids) < n:
                time.sleep(0.2)

    # -- transport -------------------------------------------------------------------
    def _send(self, msg):
        with self._send_lock:
            self._conn.send(msg)

    def _request(self, msg, timeout=30.0) -> dict:
        rid = P.new_msg_id()
        msg["req_id"] = rid
        self._send(msg)
        with self._reply_cv:
            ok = self._reply_cv.wait_for(lambda: rid in self._replies or self._closed, timeout)
            if not ok or rid not in self._replies:
                raise TimeoutError("farm controller did not answer %s" % msg["type"])
            return self._replies.pop(rid)

    def _add_callback(self, rec: _TaskRecord, fn):
        with self._rec_lock:
            if not rec.event.is_set():
                rec.callbacks.append(fn)
                return
        fn(rec)

    def _recv_loop(self):
        while True:
            try:
                msg = self._conn.recv()
            except Exception:        # EOF, or the connection closed under us by close()
                break
            t = msg.get("type")
            if t == "reply":
                with self._reply_cv:
                    self._replies[msg.get("req_id")] = msg
                    self._reply_cv.notify_all()
                continue
            if t == "engine_event":
                self.engine_events.append(msg)
                continue
            rec = self._records.get(msg.get("msg_id"))
            if rec is None:
                continue
            if "engine_id" in msg and msg["engine_id"] is not None:
                rec.engine_id = msg["engine_id"]
            if t == "assigned":
                rec.status = "assigned"
            elif t == "started":
                rec.started = msg.get("t") or P.now()
                rec.status = "running"
            elif t == "stream":
                if msg["name"] == "stdout":
                    rec.stdout += msg["text"]
                else:
                    rec.stderr += msg["text"]
            elif t == "datapub":
                d = dict(rec.data)
                d.update(P.loads(msg["data"]))
                rec.data = d
            elif t == "result":
                rec.completed = msg.get("t") or P.now()
                if msg.get("ok"):
                    try:
                        rec.value = P.loads(msg["value"])
                        rec.ok = True
                    except Exception as e:   # noqa: BLE001
                        rec.ok, rec.error = False, RemoteError("DeserializationError", str(e))
                else:
                    cls = {"TaskAborted": TaskAborted, "EngineError": EngineError}.get(msg.get("ename"), RemoteError)
                    rec.ok = False
                    rec.error = cls(msg.get("ename", "Error"), msg.get("evalue", ""), msg.get("traceback", ""),
                                    rec.engine_id)
                rec.status = "done" if rec.ok else ("aborted" if isinstance(rec.error, TaskAborted) else "error")
                with self._rec_lock:
                    rec.event.set()
                    cbs, rec.callbacks = rec.callbacks, []
                for cb in cbs:
                    try:
                        cb(rec)
                    except Exception:
                        pass
        self._closed = True
        with self._reply_cv:
            self._reply_cv.notify_all()
        for rec in list(self._records.values()):       # fail everything still pending
            if not rec.event.is_set():
                rec.ok = False
                rec.error = EngineError("EngineError", "lost connection to the farm controller")
                rec.status = "error"
                rec.event.set()

    def _submit(self, target: Optional[int], kind: str, payload) -> str:
        mid = P.new_msg_id()
        rec = _TaskRecord(mid)
        with self._rec_lock:
            self._records[mid] = rec
        self._send({"type": "submit", "msg_id": mid, "target": target, "kind": kind, "payload": P.dumps(payload)})
        return mid

    # -- public API ---------------------------------------------------------------------
    @property
    def ids(self) -> List[int]:
        if not self._closed:
            try:
                self._ids = self._request({"type": "ids"}).get("ids", self._ids)
            except TimeoutError:
                pass
        return list(self._ids)

    def __len__(self):
        return len(self.ids)

    def __getitem__(self, key) -> DirectView:
        ids = self.ids
        if isinstance(key, int):
            if key not in ids and not (-len(ids) <= key < 0):
                raise IndexError("no engine %d" % key)
            return DirectView(self, ids[key] if key < 0 else key)
        if isinstance(key, slice):
            return DirectView(self, ids[key])
        return DirectView(self, list(key))

    def direct_view(self, targets="all") -> DirectView:
        return DirectView(self, self.ids if targets == "all" else targets)

    def load_balanced_view(self, targets=None) -> LoadBalancedView:
        return LoadBalancedView(self, targets)

    @property
    def outstanding(self):
        return {m for m, r in self._records.items() if not r.event.is_set()}

    @property
    def results(self):
        return {m: r.value for m, r in self._records.items() if r.event.is_set() and r.ok}

    @property
    def metadata(self):
        return {m: AsyncResult(self, [m], True).metadata for m in self._records}

    def wait(self, jobs=None, timeout=-1) -> bool:
        if jobs is None:
            ids = list(self.outstanding)
        else:
            jobs = jobs if isinstance(jobs, (list, tuple, set)) else [jobs]
            ids = []
            for j in jobs:
                ids.extend(j.msg_ids if isinstance(j, AsyncResult) else [j])
        return AsyncResult(self, ids, single=False).wait(timeout)

    def abort(self, jobs=None, grace: Optional[float] = None):
        if jobs is None:
            ids = list(self.outstanding)
        else:
            jobs = jobs if isinstance(jobs, (list, tuple, set)) else [jobs]
            ids = []
            for j in jobs:
                ids.extend(j.msg_ids if isinstance(j, AsyncResult) else [j])
        self._request({"type": "abort", "msg_ids": ids, "grace": grace})

    def queue_status(self, verbose=False):
        return self._request({"type": "queue_status"})["status"]

    def restart_engines(self, engine_ids: Iterable[int]):
        self._request({"type": "restart", "engine_ids": list(engine_ids)})

    def shutdown(self, hub: bool = True, block: bool = True):
        if hub and not self._closed:
            try:
                self._request({"type": "shutdown"})
            except TimeoutError:
                pass
        self.close()

    def close(self):
        if self._conn is not None:
            try:
                self._conn.close()
            except Exception:
                pass
        self._closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
