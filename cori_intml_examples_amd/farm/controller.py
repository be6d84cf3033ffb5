"""Farm controller: task hub + engine supervisor for one MI355X node (``ipcontroller``
analogue, ``startCluster.sh:14``).

* Accepts engines and clients on an authenticated Unix socket (``protocol.py``).
* Direct tasks (``client[i].apply/execute/push/pull``) queue FIFO per engine;
  load-balanced tasks (``load_balanced_view().apply``) go to the least-loaded idle engine
  (IPyParallel's default "leastload" scheme, one task in flight per engine).
* Streams each task's ``started`` / stdout / stderr / ``publish_data`` / result back to
  the submitting client as they happen.
* Supervises the engine processes it spawned (one per GPU, ``HIP_VISIBLE_DEVICES``
  pinned): an engine that dies fails its running task with ``EngineError`` and is
  restarted; ``abort`` removes queued tasks, interrupts running ones and hard-kills the
  engine after a grace period (the reference's Stop/Restart were stubs,
  ``hpo_widgets.py:352-364,386-391``).
"""
from __future__ import annotations

import argparse
import collections
import os
import signal
import subprocess
import sys
import threading
import time
from multiprocessing.connection import Listener, wait
from typing import Any, Deque, Dict, List, Optional

from . import protocol as P


class _Task:
    __slots__ = ("msg_id", "client", "target", "kind", "payload", "engine", "state", "abort_deadline",
                 "interrupt_at", "submitted")

    def __init__(self, msg_id, client, target, kind, payload):
        self.msg_id, self.client, self.target, self.kind, self.payload = msg_id, client, target, kind, payload
        self.engine: Optional[int] = None
        self.state = "queued"         # queued | running | done
        self.abort_deadline: Optional[float] = None
        self.interrupt_at: Optional[float] = None
        self.submitted = time.time()


class _EngineRec:
    def __init__(self, eid: int, gpu: Optional[str]):
        self.eid, self.gpu = eid, gpu
        self.proc: Optional[subprocess.Popen] = None
        self.conn = None
        self.current: Optional[str] = None
        self.queue: Deque[str] = collections.deque()
        self.restarts = 0
        self.started_at = 0.0
        self.stats: Dict[str, Any] = {}     # last resource telemetry from the engine


def _remap_gpu(idx: str) -> str:
    """The physical device behind logical GPU ``idx``: ``INTML_FARM_GPU_REMAP`` ("1:0,2:0" or
    "*:0") remaps indices at the very last step, the engine's HIP_VISIBLE_DEVICES -- the
    one-GPU rehearsal of a one-engine-per-GPU farm (every other decision, the engines' DP
    environment included, sees distinct GPUs).  Unset: the identity."""
    spec = os.environ.get("INTML_FARM_GPU_REMAP", "")
    for item in filter(None, (x.strip() for x in spec.split(","))):
        src, _, dst = item.partition(":")
        if dst and (src == "*" or src == idx):
            return dst
    return idx


class Controller:
    def __init__(self, cluster_id: str, n_engines: int, gpus: Optional[List[str]] = None,
                 engine_env: Optional[Dict[str, str]] = None, abort_grace: float = 10.0,
                 restart: bool = True, dp_port: Optional[int] = None, python: str = sys.executable):
        self.info = P.new_connection_info(cluster_id)
        self.n = int(n_engines)
        self.gpus = gpus
        self.engine_env = dict(engine_env or {})
        self.abort_grace = float(abort_grace)
        self.restart = restart
        self.python = python
        self.dp_port = dp_port or (29500 + (os.getpid() % 2000))
        self.listener = Listener(self.info["address"], family="AF_UNIX", authkey=P.authkey(self.info))
        self.info["n_engines"] = self.n
        self.info["dp_port"] = self.dp_port
        self._pending: Deque = collections.deque()
        self._lock = threading.Lock()
        self.engines: Dict[int, _EngineRec] = {}
        self.clients: List[Any] = []
        self.tasks: Dict[str, _Task] = {}
        self.lb_queue: Deque[str] = collections.deque()
        self.running = True
        self._accept_thread = threading.Thread(target=self._accept_loop, daemon=True, name="farm-accept")

    # ------------------------------------------------------------------ engines
    def _engine_env(self, eid: int) -> Dict[str, str]:
        env = dict(os.environ)
        env.update(self.engine_env)
        if self.gpus is not None:
            env["HIP_VISIBLE_DEVICES"] = _remap_gpu(str(self.gpus[eid % len(self.gpus)]))
        # DP rank environment: %%px + hvd.init() turns the engines into one RCCL job
        env.update({"RANK": str(eid), "WORLD_SIZE": str(self.n), "LOCAL_RANK": "0",
                    "LOCAL_WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(self.dp_port),
                    "INTML_FARM_ENGINE": str(eid), "INTML_FARM_CLUSTER": self.info["cluster_id"]})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if self.gpus is not None and len(set(self.gpus[e % len(self.gpus)] for e in range(self.n))) < self.n:
            # engines share a GPU: RCCL refuses two ranks on one device, so a %%px data-parallel
            # job over these engines runs the RCCL-free xGMI plane -- on EVERY engine (every rank
            # must pick the same plane)
            env.setdefault("INTML_COMM", "xgmi")
        return env

    def _spawn(self, eid: int):
        rec = self.engines.setdefault(eid, _EngineRec(eid, None if self.gpus is None else
                                                      str(self.gpus[eid % len(self.gpus)])))
        # -c (not -m): the engine module must be the imported one so publish_data sees it
        cmd = [self.python, "-c", "from cori_intml_examples_amd.farm.engine import main; main()",
               "--connection-file", P.connection_file(self.info["cluster_id"]), "--engine-id", str(eid)]
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = self._engine_env(eid)
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        rec.proc = subprocess.Popen(cmd, env=env, stdin=subprocess.DEVNULL)
        rec.conn = None
        rec.started_at = time.time()

    # ------------------------------------------------------------------ sockets
    def _accept_loop(self):
        while self.running:
            try:
                c = self.listener.accept()
            except Exception:
                if not self.running:
                    return
                continue
            with self._lock:
                self._pending.append(c)

    def _conns(self):
        out = list(self.clients)
        out += [e.conn for e in self.engines.values() if e.conn is not None]
        return out

    def _send(self, conn, msg):
        if conn is None:
            return
        try:
            conn.send(msg)
        except Exception:
            pass

    # ------------------------------------------------------------------ main loop
    def serve(self):
        P.write_connection_file(self.info)
        self._accept_thread.start()
        for eid in range(self.n):
            self._spawn(eid)
        try:
            while self.running:
                self._drain_pending()
                conns = self._conns()
                ready = wait(conns, timeout=0.05) if conns else (time.sleep(0.05) or [])
                for c in ready:
                    try:
                        msg = c.recv()
                    except (EOFError, OSError):
                        self._disconnect(c)
                        continue
                    self._handle(c, msg)
                self._supervise()
                self._schedule()
        finally:
            self._teardown()

    def _drain_pending(self):
        while True:
            with self._lock:
                if not self._pending:
                    return
                c = self._pending.popleft()
            try:
                if not c.poll(5.0):
                    c.close()
                    continue
                hello = c.recv()
            except Exception:
                continue
            if hello.get("role") == "engine":
                eid = int(hello["engine_id"])
                rec = self.engines.get(eid)
                if rec is None:
                    c.close()
                    continue
                rec.conn = c
                self._broadcast({"type": "engine_event", "event": "registered", "engine_id": eid})
            else:
                self.clients.append(c)
                self._send(c, {"type": "reply", "req_id": hello.get("req_id"), "ids": self._ids(),
                               "info": {k: v for k, v in self.info.items() if k != "authkey"}})

    def _ids(self):
        return sorted(e.eid for e in self.engines.values() if e.conn is not None)

    def _broadcast(self, msg):
        for c in list(self.clients):
            self._send(c, msg)

    def _engine_of_conn(self, c) -> Optional[_EngineRec]:
        for e in self.engines.values():
            if e.conn is c:
                return e
        return None

    def _disconnect(self, c):
        e = self._engine_of_conn(c)
        if e is not None:
            e.conn = None
            return          # process death is handled by _supervise
        if c in self.clients:
            self.clients.remove(c)
            # orphaned queued tasks of that client are dropped
            for t in list(self.tasks.values()):
                if t.client is c and t.state == "queued":
                    self._forget_queued(t)

    def _forget_queued(self, t: _Task):
        if t.target is None:
            if t.msg_id in self.lb_queue:
                self.lb_queue.remove(t.msg_id)
        else:
            rec = self.engines.get(t.target)
            if rec is not None and t.msg_id in rec.queue:
                rec.queue.remove(t.msg_id)
        t.state = "done"
        self.tasks.pop(t.msg_id, None)

    # ------------------------------------------------------------------ messages
    def _handle(self, c, msg):
        t = msg.get("type")
        e = self._engine_of_conn(c)
        if e is not None:
            self._handle_engine(e, msg)
            return
        if t == "submit":
            self._submit(c, msg)
        elif t == "ids":
            self._send(c, {"type": "reply", "req_id": msg.get("req_id"), "ids": self._ids()})
        elif t == "queue_status":
            st = {e.eid: dict({k: v for k, v in e.stats.items() if k.endswith("_bytes") or k == "t"},
                              queue=len(e.queue), running=e.current, restarts=e.restarts,
                              pid=e.proc.pid if e.proc else None, gpu=e.gpu)
                  for e in self.engines.values()}
            st["unassigned"] = len(self.lb_queue)
            self._send(c, {"type": "reply", "req_id": msg.get("req_id"), "status": st})
        elif t == "abort":
            for mid in msg.get("msg_ids", []):
                self._abort(mid, msg.get("grace"))
            self._send(c, {"type": "reply", "req_id": msg.get("req_id")})
        elif t == "restart":
            for eid in msg.get("engine_ids", []):
                self._kill_engine(int(eid), "restart requested")
            self._send(c, {"type": "reply", "req_id": msg.get("req_id")})
        elif t == "shutdown":
            self._send(c, {"type": "reply", "req_id": msg.get("req_id")})
            self.running = False

    def _submit(self, c, msg):
        task = _Task(msg["msg_id"], c, msg.get("target"), msg["kind"], msg.get("payload"))
        self.tasks[task.msg_id] = task
        if task.target is None:
            self.lb_queue.append(task.msg_id)
        else:
            rec = self.engines.get(int(task.target))
            if rec is None:
                self._finish(task, {"type": "result", "msg_id": task.msg_id, "ok": False,
                                    "ename": "IndexError", "evalue": "no engine %s" % task.target,
                                    "t": P.now()})
                return
            rec.queue.append(task.msg_id)

    def _handle_engine(self, e: _EngineRec, msg):
        if msg.get("type") == "stats":
            e.stats = dict(msg.get("stats") or {}, t=time.time())
            return
        mid = msg.get("msg_id")
        task = self.tasks.get(mid)
        if task is None:
            return
        t = msg["type"]
        if t == "result":
            msg["engine_id"] = e.eid
            if e.current == mid:
                e.current = None
            self._finish(task, msg)
        else:
            msg["engine_id"] = e.eid
            self._send(task.client, msg)

    def _finish(self, task: _Task, msg):
        task.state = "done"
        self.tasks.pop(task.msg_id, None)
        self._send(task.client, msg)

    # ------------------------------------------------------------------ scheduling
    def _dispatch(self, rec: _EngineRec, mid: str):
        task = self.tasks[mid]
        task.engine, task.state = rec.eid, "running"
        rec.current = mid
        try:
            rec.conn.send({"type": "task", "msg_id": mid, "kind": task.kind, "payload": task.payload})
        except Exception:
            rec.current = None
            task.state = "queued"
            (self.lb_queue.appendleft if task.target is None else rec.queue.appendleft)(mid)
            return
        self._send(task.client, {"type": "assigned", "msg_id": mid, "engine_id": rec.eid})

    def _schedule(self):
        idle = [e for e in self.engines.values() if e.conn is not None and e.current is None]
        for rec in idle:                       # direct queues first (FIFO per engine)
            if rec.queue:
                self._dispatch(rec, rec.queue.popleft())
        idle = sorted((e for e in self.engines.values() if e.conn is not None and e.current is None
                       and not e.queue), key=lambda e: e.eid)
        for rec in idle:
            if not self.lb_queue:
                break
            self._dispatch(rec, self.lb_queue.popleft())

    # ------------------------------------------------------------------ abort / supervise
    def _abort(self, mid: str, grace=None):
        task = self.tasks.get(mid)
        if task is None:
            return
        if task.state == "queued":
            self._forget_queued(task)
            self._send(task.client, {"type": "result", "msg_id": mid, "ok": False, "ename": "TaskAborted",
                                     "evalue": "aborted before it started", "t": P.now()})
            return
        rec = self.engines.get(task.engine)
        if rec is not None:
            # staged cancel: cooperative flag now (training stops at the next batch end),
            # KeyboardInterrupt at half the grace period, engine kill at the full grace
            g = self.abort_grace if grace is None else float(grace)
            self._send(rec.conn, {"type": "interrupt", "msg_id": mid, "cooperative_only": True})
            task.interrupt_at = time.time() + 0.5 * g
            task.abort_deadline = time.time() + g

    def _kill_engine(self, eid: int, why: str):
        rec = self.engines.get(eid)
        if rec is None or rec.proc is None:
            return
        try:
            rec.proc.kill()
        except Exception:
            pass

    def _supervise(self):
        now = time.time()
        for t in list(self.tasks.values()):
            if t.state == "running" and t.interrupt_at is not None and now > t.interrupt_at:
                t.interrupt_at = None
                rec = self.engines.get(t.engine)
                if rec is not None:
                    self._send(rec.conn, {"type": "interrupt", "msg_id": t.msg_id})
            if t.state == "running" and t.abort_deadline is not None and now > t.abort_deadline:
                t.abort_deadline = None
                self._kill_engine(t.engine, "abort grace expired")
        for rec in list(self.engines.values()):
            if rec.proc is None or rec.proc.poll() is None:
                continue
            code = rec.proc.returncode
            if rec.conn is not None:
                try:
                    rec.conn.close()
                except Exception:
                    pass
                rec.conn = None
            if rec.current is not None:
                task = self.tasks.get(rec.current)
                rec.current = None
                if task is not None:
                    aborted = task.abort_deadline is not None or code in (-signal.SIGKILL,)
                    self._finish(task, {"type": "result", "msg_id": task.msg_id, "ok": False,
                                        "ename": "TaskAborted" if aborted else "EngineError",
                                        "evalue": "engine %d exited with code %s while running the task"
                                                  % (rec.eid, code), "engine_id": rec.eid, "t": P.now()})
            self._broadcast({"type": "engine_event", "event": "died", "engine_id": rec.eid, "code": code})
            if self.running and self.restart:
                rec.restarts += 1
                self._spawn(rec.eid)
            else:
                rec.proc = None

    def _teardown(self):
        self.running = False
        for rec in self.engines.values():
            self._send(rec.conn, {"type": "shutdown"})
        deadline = time.time() + 5
        for rec in self.engines.values():
            if rec.proc is None:
                continue
            try:
                rec.proc.wait(timeout=max(0.1, deadline - time.time()))
            except Exception:
                rec.proc.kill()
        for t in list(self.tasks.values()):
            self._send(t.client, {"type": "result", "msg_id": t.msg_id, "ok": False, "ename": "EngineError",
                                  "evalue": "cluster shut down", "t": P.now()})
        try:
            self.listener.close()
        except Exception:
            pass
        for p in (self.info["address"], P.connection_file(self.info["cluster_id"])):
            try:
                os.remove(p)
            except OSError:
                pass


def main(argv=None):
    ap = argparse.ArgumentParser(description="intml farm controller (one node)")
    ap.add_argument("--cluster-id", default="default")
    ap.add_argument("-n", "--n-engines", type=int, default=None, help="engines (default: one per GPU)")
    ap.add_argument("--gpus", default=None, help="comma list of GPU indices to pin engines to ('none' = unpinned)")
    ap.add_argument("--abort-grace", type=float, default=10.0)
    ap.add_argument("--no-restart", action="store_true")
    a = ap.parse_args(argv)
    from .cluster import detect_gpus
    gpus = None
    if a.gpus and a.gpus != "none":
        gpus = a.gpus.split(",")
    elif a.gpus is None:
        n_gpu = detect_gpus()
        gpus = [str(i) for i in range(n_gpu)] if n_gpu else None
    n = a.n_engines or (len(gpus) if gpus else 1)
    ctl = Controller(a.cluster_id, n, gpus, abort_grace=a.abort_grace, restart=not a.no_restart)
    signal.signal(signal.SIGTERM, lambda *_: setattr(ctl, "running", False))
    ctl.serve()


if __name__ == "__main__":
    main()
