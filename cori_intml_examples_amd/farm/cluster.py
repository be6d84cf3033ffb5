"""Cluster bring-up on one MI355X node: the ``startCluster.sh`` equivalent.

The reference starts one ``ipcontroller`` on the head node, sleeps 30 s, then
``srun ipengine`` once per SLURM task (``startCluster.sh:8-18``), with the cluster id
``cori_${SLURM_JOB_ID}`` that notebooks rebuild to connect (``DistTrain_mnist.ipynb:68-69``).
Here one controller process spawns one engine per GPU (``HIP_VISIBLE_DEVICES`` pinned)
and returns as soon as every engine has registered -- no fixed sleep.

    python -m cori_intml_examples_amd.farm.cluster start [-n 8] [--cluster-id ID] [--daemon]
    python -m cori_intml_examples_amd.farm.cluster stop  [--cluster-id ID]
    python -m cori_intml_examples_amd.farm.cluster status [--cluster-id ID]

The default cluster id is ``intml_${SLURM_JOB_ID}`` when running under SLURM, else
``intml_<user>``.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import signal
import subprocess
import sys
import time
from typing import List, Optional

from . import protocol as P


def default_cluster_id() -> str:
    job = os.environ.get("SLURM_JOB_ID")
    if job:
        return "intml_%s" % job
    try:
        import getpass
        return "intml_%s" % getpass.getuser()
    except Exception:
        return "intml_%d" % os.getuid()


def detect_gpus() -> int:
    """Number of visible GPUs without initialising HIP (KFD topology, honouring
    ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES``)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    n = 0
    for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            with open(p) as f:
                if int(f.read().strip() or 0) != 0:
                    n += 1
        except (OSError, ValueError):
            pass
    return n


class Cluster:
    """A running farm (controller subprocess + its engines)."""

    def __init__(self, cluster_id: str, proc: Optional[subprocess.Popen] = None):
        self.cluster_id = cluster_id
        self.proc = proc

    def client(self, timeout: float = 60):
        from .client import Client
        return Client(cluster_id=self.cluster_id, timeout=timeout)

    def wait_ready(self, n_engines: int, timeout: float = 120) -> None:
        from .client import Client
        deadline = time.time() + timeout
        while True:
            if self.proc is not None and self.proc.poll() is not None:
                raise RuntimeError("farm controller exited with code %s" % self.proc.returncode)
            try:
                with Client(cluster_id=self.cluster_id, timeout=max(1.0, deadline - time.time())) as c:
                    if len(c.ids) >= n_engines:
                        return
            except TimeoutError:
                pass
            if time.time() > deadline:
                raise TimeoutError("farm %r: engines did not register within %.0fs" % (self.cluster_id, timeout))
            time.sleep(0.2)

    def stop(self, timeout: float = 15) -> None:
        from .client import Client
        try:
            with Client(cluster_id=self.cluster_id, timeout=2) as c:
                c.shutdown()
        except Exception:
            pass
        if self.proc is not None:
            try:
                self.proc.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()


def start_cluster(n_engines: Optional[int] = None, cluster_id: Optional[str] = None,
                  gpus: Optional[List[int]] = None, cpu_only: bool = False, abort_grace: float = 10.0,
                  restart: bool = True, timeout: float = 120, env: Optional[dict] = None,
                  log_file: Optional[str] = None) -> Cluster:
    """Start a controller + engines and wait until they are all registered.

    ``gpus``: GPU indices to pin engines to round-robin (default: every visible GPU, one
    engine each).  ``cpu_only``: unpinned engines with ``INTML_DEVICE=cpu`` (tests, or a
    node without GPUs)."""
    cluster_id = cluster_id or default_cluster_id()
    if gpus is None and not cpu_only:
        g = detect_gpus()
        gpus = list(range(g)) if g else None
    if n_engines is None:
        n_engines = len(gpus) if gpus else 1
    cmd = [sys.executable, "-c", "from cori_intml_examples_amd.farm.controller import main; main()",
           "--cluster-id", cluster_id,
           "-n", str(n_engines), "--abort-grace", str(abort_grace)]
    cmd += ["--gpus", ",".join(str(x) for x in gpus)] if gpus else ["--gpus", "none"]
    if not restart:
        cmd.append("--no-restart")
    e = dict(os.environ)
    e.update(env or {})
    if cpu_only:
        e["INTML_DEVICE"] = "cpu"
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    e["PYTHONPATH"] = root + (os.pathsep + e["PYTHONPATH"] if e.get("PYTHONPATH") else "")
    try:                                   # a stale file from a dead cluster would mislead clients
        os.remove(P.connection_file(cluster_id))
    except OSError:
        pass
    out = open(log_file, "ab") if log_file else None
    proc = subprocess.Popen(cmd, env=e, stdin=subprocess.DEVNULL, stdout=out, stderr=out,
                            start_new_session=True)
    cl = Cluster(cluster_id, proc)
    cl.wait_ready(n_engines, timeout)
    return cl


def main(argv=None):
    ap = argparse.ArgumentParser(description="one-node farm (startCluster.sh equivalent)")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("start")
    s.add_argument("-n", "--n-engines", type=int, default=None)
    s.add_argument("--cluster-id", default=None)
    s.add_argument("--gpus", default=None, help="comma list (default: all visible)")
    s.add_argument("--cpu", action="store_true", help="CPU-only engines")
    s.add_argument("--daemon", action="store_true", help="return once ready, leave the farm running")
    s.add_argument("--log-file", default=None)
    for name in ("stop", "status"):
        p = sub.add_parser(name)
        p.add_argument("--cluster-id", default=None)
    a = ap.parse_args(argv)
    cid = a.cluster_id or default_cluster_id()
    if a.cmd == "start":
        gpus = [int(x) for x in a.gpus.split(",")] if a.gpus else None
        cl = start_cluster(a.n_engines, cid, gpus, cpu_only=a.cpu, log_file=a.log_file)
        with cl.client() as c:
            print("cluster %s: %d engines %s" % (cid, len(c.ids), c.ids), flush=True)
        if a.daemon:
            return
        try:
            signal.signal(signal.SIGTERM, lambda *_: (_ for _ in ()).throw(KeyboardInterrupt()))
            cl.proc.wait()
        except KeyboardInterrupt:
            cl.stop()
    elif a.cmd == "stop":
        Cluster(cid).stop()
    else:
        from .client import Client
        with Client(cluster_id=cid, timeout=5) as c:
            print(json.dumps(c.queue_status(), indent=1, default=str))


if __name__ == "__main__":
    main()
