"""Control-plane plumbing shared by the farm's controller, engines and clients.

The reference's control plane is IPyParallel over ZeroMQ/TCP, with the controller bound
to the Aries NIC and rendezvous through the IPython profile dir + ``--cluster-id``
(``startCluster.sh:8-18``).  On one MI355X node the farm uses local
Unix-domain sockets (``multiprocessing.connection`` framing, HMAC authkey challenge) with
cloudpickle payloads.  A cluster is found by id through a JSON connection file
``<runtime_dir>/<cluster_id>.json`` (mode 0600: it holds the authkey).

Message kinds (dicts with a ``type`` key):
  client -> controller   hello, submit, abort, ids, queue_status, shutdown, restart
  controller -> client   reply, started, stream, datapub, result, engine_event
  engine -> controller   hello, started, stream, datapub, result
  controller -> engine   task, interrupt, shutdown
"""
from __future__ import annotations

import datetime as _dt
import json
import os
import secrets
import tempfile
import uuid
from typing import Any, Dict

import cloudpickle


class InsecurePathError(PermissionError):
    """A runtime directory / connection file another user could have planted or modified."""


def _check_private(path: str, want_dir: bool) -> None:
    """Refuse ``path`` unless it is a real (non-symlink) file/directory owned by this user
    with no group/other permission bits: the connection file carries the authkey and the
    socket address whose payloads are unpickled."""
    st = os.lstat(path)
    import stat as _stat
    kind_ok = _stat.S_ISDIR(st.st_mode) if want_dir else _stat.S_ISREG(st.st_mode)
    if not kind_ok:
        raise InsecurePathError("%s is not a regular %s (symlink?)" % (path, "directory" if want_dir else "file"))
    if st.st_uid != os.getuid():
        raise InsecurePathError("%s is owned by uid %d, not %d" % (path, st.st_uid, os.getuid()))
    if st.st_mode & 0o077:
        raise InsecurePathError("%s has mode %o: group/other access is not allowed" % (path, st.st_mode & 0o777))


def runtime_dir() -> str:
    """Per-user private directory for connection files and sockets: ``$INTML_FARM_DIR``,
    else ``$XDG_RUNTIME_DIR/intml-farm``, else ``/tmp/intml-farm-<uid>``; checked to be
    ours and private (a pre-created world-writable dir is refused)."""
    d = os.environ.get("INTML_FARM_DIR")
    if not d:
        xdg = os.environ.get("XDG_RUNTIME_DIR")
        if xdg and os.path.isdir(xdg):
            d = os.path.join(xdg, "intml-farm")
        else:
            d = os.path.join(tempfile.gettempdir(), "intml-farm-%d" % os.getuid())
    os.makedirs(d, mode=0o700, exist_ok=True)
    _check_private(d, want_dir=True)
    return d


def connection_file(cluster_id: str) -> str:
    return os.path.join(runtime_dir(), "%s.json" % (cluster_id or "default"))


def new_connection_info(cluster_id: str) -> Dict[str, Any]:
    # AF_UNIX paths are limited to ~107 bytes: keep the socket name short
    sock = os.path.join(runtime_dir(), "c-%s.sock" % uuid.uuid4().hex[:12])
    return {"cluster_id": cluster_id or "default", "address": sock, "authkey": secrets.token_hex(16),
            "pid": os.getpid(), "created": now().isoformat()}


def write_connection_file(info: Dict[str, Any]) -> str:
    path = connection_file(info["cluster_id"])
    tmp = path + ".tmp%d" % os.getpid()
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "w") as f:
        json.dump(info, f)
    os.replace(tmp, path)
    return path


def read_connection_file(cluster_id: str = None, path: str = None) -> Dict[str, Any]:
    path = path or connection_file(cluster_id)
    _check_private(path, want_dir=False)
    with open(path) as f:
        return json.load(f)


def authkey(info) -> bytes:
    return bytes.fromhex(info["authkey"])


def dumps(obj) -> bytes:
    return cloudpickle.dumps(obj)


def loads(b: bytes):
    # payloads only ever come from this cluster's own authenticated processes
    return cloudpickle.loads(b)


def now() -> _dt.datetime:
    return _dt.datetime.now()


def new_msg_id() -> str:
    return uuid.uuid4().hex


class RemoteError(Exception):
    """An exception raised inside an engine task (IPyParallel ``RemoteError`` analogue)."""

    def __init__(self, ename: str, evalue: str, traceback: str = "", engine_id=None):
        super().__init__("%s(%s)" % (ename, evalue))
        self.ename, self.evalue, self.traceback, self.engine_id = ename, evalue, traceback, engine_id

    def __str__(self):
        eng = "" if self.engine_id is None else "[engine %s] " % self.engine_id
        return "%s%s: %s" % (eng, self.ename, self.evalue)

    def render_traceback(self):
        return self.traceback.splitlines()


class TaskAborted(RemoteError):
    pass


class EngineError(RemoteError):
    """The engine running the task died (crash, OOM, hard kill)."""
