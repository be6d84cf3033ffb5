"""Notebook front-ends of the farm: ``%%px`` / ``%px`` and ``%ipcluster``.

* ``%%px`` runs a cell on every engine (SPMD), as the reference's DistTrain notebooks do
  (``DistTrain_mnist.ipynb:104,145,159,222,292,488,553``); stdout of each engine is
  printed with an ``[stdout:i]`` header like IPyParallel.  ``px(code)`` is the same
  thing as a plain function (scripts, tests, no IPython).
* ``%ipcluster`` starts a farm from a cell.  The reference's magic (``ipcluster_magics.py:
  12-256``) wrote three temp scripts and ran ``salloc`` + ``srun ipengine`` on Cori
  nodes; on one MI355X node the same options map to: ``-n/--num_engines`` engines
  (default: one per GPU), ``-N/--num_nodes`` must be 1, ``-m/--modules`` modules imported
  on every engine, ``-e/--env`` env vars ``K=V[,K=V]`` for the engines, ``-d/--dir``
  engines' working directory, ``-J/--name`` cluster id; ``-t/-C/-q`` (SLURM time,
  constraint, queue) are accepted and ignored.  The parser is argparse (docopt is not
  installed) with the same flags and defaults (``ipcluster_magics.py:97-130``).
"""
from __future__ import annotations

import argparse
import os
import shlex
from typing import Dict, List, Optional

from .client import Client

_CLIENT: Optional[Client] = None
_CLUSTERS: Dict[str, object] = {}


def set_client(client: Client) -> None:
    global _CLIENT
    _CLIENT = client


def _client(cluster_id=None) -> Client:
    global _CLIENT
    if _CLIENT is None or (cluster_id is not None and _CLIENT.cluster_id != cluster_id):
        _CLIENT = Client(cluster_id=cluster_id, timeout=60)
    return _CLIENT


def px(code: str, targets="all", client: Optional[Client] = None, block: bool = True, verbose: bool = True):
    """Run ``code`` on the engines (``%%px``).  Returns the AsyncResult; with ``block``
    waits, prints each engine's stdout/stderr and re-raises the first remote error."""
    c = client or _client()
    view = c.direct_view(targets)
    ar = view.execute(code, block=False)
    if not block:
        return ar
    ar.wait()
    if verbose:
        outs = ar.stdout if isinstance(ar.stdout, list) else [ar.stdout]
        errs = ar.stderr if isinstance(ar.stderr, list) else [ar.stderr]
        for t, o, e in zip(view.targets, outs, errs):
            if o:
                print("[stdout:%d] %s" % (t, o), end="" if o.endswith("\n") else "\n")
            if e:
                print("[stderr:%d] %s" % (t, e), end="" if e.endswith("\n") else "\n")
    ar.get()
    return ar


def parse_ipcluster_args(line: str) -> Dict[str, object]:
    ap = argparse.ArgumentParser(prog="%ipcluster", add_help=True)
    ap.add_argument("-N", "--num_nodes", type=int, default=1)
    ap.add_argument("-n", "--num_engines", type=int, default=None)
    ap.add_argument("-m", "--modules", nargs="*", default=None)
    ap.add_argument("-e", "--env", default=None)
    ap.add_argument("-t", "--time", default="30:00")
    ap.add_argument("-d", "--dir", default=None)
    ap.add_argument("-C", "--const", default="haswell")
    ap.add_argument("-q", "--queue", default="interactive")
    ap.add_argument("-J", "--name", default="ipyparallel")
    ap.add_argument("--cpu", action="store_true", help="CPU-only engines")
    a = vars(ap.parse_args(shlex.split(line)))
    return a


def ipcluster(line: str = ""):
    """Start a farm from options (``%ipcluster`` line magic).  Returns the Client."""
    from .cluster import start_cluster
    a = parse_ipcluster_args(line)
    if a["num_nodes"] != 1:
        raise ValueError("the farm runs on one node (got --num_nodes %d)" % a["num_nodes"])
    env = {}
    if a["env"]:
        for kv in a["env"].split(","):
            k, _, v = kv.partition("=")
            env[k.strip()] = v
    cl = start_cluster(a["num_engines"], cluster_id=a["name"], cpu_only=a["cpu"], env=env)
    _CLUSTERS[a["name"]] = cl
    c = cl.client()
    if a["dir"]:
        c[:].execute("import os; os.chdir(%r)" % os.path.expanduser(a["dir"]), block=True)
    if a["modules"]:
        c[:].execute("\n".join("import %s" % m for m in a["modules"]), block=True)
    set_client(c)
    print("cluster %s: %d engines" % (a["name"], len(c.ids)))
    return c


def stop_clusters():
    for cl in list(_CLUSTERS.values()):
        cl.stop()
    _CLUSTERS.clear()


def load_ipython_extension(ip):
    """``%load_ext cori_intml_examples_amd.farm.magics`` registers %%px, %px, %ipcluster."""
    from IPython.core.magic import Magics, cell_magic, line_magic, magics_class

    @magics_class
    class FarmMagics(Magics):
        @cell_magic
        def px(self, line, cell):
            targets = "all"
            if line.strip().startswith("--targets"):
                spec = line.split(None, 1)[1]
                targets = eval(spec, {"__builtins__": {}}, {})   # e.g. "[0,1]" or "0"
            px(cell, targets=targets)

        @line_magic("px")
        def px_line(self, line):
            px(line)

        @line_magic
        def ipcluster(self, line):
            return ipcluster(line)

    ip.register_magics(FarmMagics)


try:        # auto-register when imported inside IPython, as ipcluster_magics.py:254-256 does
    from IPython import get_ipython as _gi      # noqa: F401
    _ip = _gi()
    if _ip is not None:
        load_ipython_extension(_ip)
except ImportError:
    pass
