"""Headless notebook runner: execute a ``.ipynb``'s code cells in order, in one namespace,
without Jupyter or IPython (neither is installed on the MI355X nodes).

IPython syntax used by the workflow notebooks is translated:
  ``%%px [--targets N|a:b] [--noblock]``  -> ``farm.magics.px(cell, targets=...)`` on the
                                            current farm client (SPMD over the engines)
  ``%%time`` / ``%time stmt``            -> run and print ``Wall time: ...``
  ``%%bash`` / ``%%sh``                  -> run with bash (skipped with ``skip_shell``)
  ``%ipcluster ...``                     -> ``farm.magics.ipcluster(...)``
  ``%matplotlib ...``, ``%load_ext ...``, other line magics -> ignored
  ``!cmd``                              -> run with the shell (skipped with ``skip_shell``)
  a trailing bare expression            -> printed (the cell's displayed value)

    python -m cori_intml_examples_amd.utils.nbrun notebooks/DistTrain_mnist.ipynb [--env K=V ...]

The notebooks read their problem sizes from ``NB_*`` environment variables (defaults: the
reference's sizes), so CI executes every notebook end to end at tiny sizes.
"""
from __future__ import annotations

import argparse
import ast
import json
import os
import shlex
import subprocess
import sys
import time
from typing import Any, Dict, List, Optional


def _targets(spec: Optional[str]):
    if spec is None or spec == "all":
        return "all"
    if ":" in spec:
        a, b = spec.split(":")
        return list(range(int(a or 0), int(b)))
    if "," in spec:
        return [int(v) for v in spec.split(",")]
    return int(spec)


def translate(source: str, skip_shell: bool = False) -> str:
    """IPython cell source -> plain Python source."""
    lines = source.splitlines()
    if not lines:
        return ""
    head = lines[0].strip()
    body = "\n".join(lines[1:])
    if head.startswith("%%px"):
        args = shlex.split(head[4:])
        p = argparse.ArgumentParser(prog="%%px", add_help=False)
        p.add_argument("--targets", "-t", default=None)
        p.add_argument("--noblock", action="store_true")
        p.add_argument("--block", action="store_true")
        a, _ = p.parse_known_args(args)
        return "__nb_px__(%r, targets=%r, block=%r)" % (body, _targets(a.targets), not a.noblock)
    if head.startswith("%%time"):
        return "__nb_t0__ = __nb_time__.time()\n%s\nprint('Wall time: %%.2f s' %% (__nb_time__.time() - __nb_t0__))" % (
            translate(body, skip_shell))
    if head.startswith("%%bash") or head.startswith("%%sh"):
        return "" if skip_shell else "__nb_sh__(%r)" % body
    if head.startswith("%%"):
        return ""                                  # other cell magics: not supported headless
    out: List[str] = []
    for ln in lines:
        s = ln.lstrip()
        ind = ln[:len(ln) - len(s)]
        if s.startswith("!"):
            out.append(ind + ("pass" if skip_shell else "__nb_sh__(%r)" % s[1:]))
        elif s.startswith("%ipcluster"):
            out.append(ind + "__nb_ipcluster__(%r)" % s[len("%ipcluster"):].strip())
        elif s.startswith("%time "):
            out.append(ind + "__nb_t0__ = __nb_time__.time(); %s; print('Wall time: %%.2f s' %% "
                             "(__nb_time__.time() - __nb_t0__))" % s[6:])
        elif s.startswith("%"):
            out.append(ind + "pass")               # %matplotlib, %load_ext, ...
        else:
            out.append(ln)
    return "\n".join(out)


def _sh(cmd: str) -> None:
    r = subprocess.run(["bash", "-c", cmd], capture_output=True, text=True)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)


def _exec_cell(code: str, ns: Dict[str, Any], name: str) -> None:
    tree = ast.parse(code, filename=name)
    last = None
    if tree.body and isinstance(tree.body[-1], ast.Expr):
        last = ast.Expression(tree.body.pop().value)
    exec(compile(tree, name, "exec"), ns)
    if last is not None:
        val = eval(compile(last, name, "eval"), ns)
        if val is not None:
            print(repr(val))


def run_notebook(path: str, env: Optional[Dict[str, str]] = None, skip_shell: bool = True,
                 verbose: bool = True) -> Dict[str, Any]:
    """Execute every code cell of ``path``; returns the final namespace.  Raises (with the
    cell index) on the first failing cell."""
    with open(path) as f:
        nb = json.load(f)
    if env:
        os.environ.update(env)
    nb_dir = os.path.dirname(os.path.abspath(path))
    root = os.path.dirname(nb_dir)
    for p in (root, nb_dir):
        if p not in sys.path:
            sys.path.insert(0, p)
    from ..farm import magics

    def _px(code, targets="all", block=True):
        return magics.px(code, targets=targets, block=block)

    ns: Dict[str, Any] = {"__name__": "__main__", "__nb_px__": _px, "__nb_sh__": _sh,
                          "__nb_ipcluster__": magics.ipcluster, "__nb_time__": time}
    cwd = os.getcwd()
    os.chdir(nb_dir)
    try:
        for i, cell in enumerate(nb.get("cells", [])):
            if cell.get("cell_type") != "code":
                continue
            src = "".join(cell.get("source", []))
            code = translate(src, skip_shell=skip_shell)
            if not code.strip():
                continue
            if verbose:
                print("---- [cell %d] %s" % (i, src.strip().splitlines()[0][:80] if src.strip() else ""), flush=True)
            try:
                _exec_cell(code, ns, "<%s cell %d>" % (os.path.basename(path), i))
            except Exception as e:
                raise RuntimeError("%s: cell %d failed: %s: %s" % (path, i, type(e).__name__, e)) from e
            sys.stdout.flush()
    finally:
        os.chdir(cwd)
        cleanup = ns.get("__nb_cleanup__")
        if callable(cleanup):
            cleanup()
    return ns


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Run a notebook's code cells headless")
    ap.add_argument("notebook")
    ap.add_argument("--env", action="append", default=[], help="K=V set before running (e.g. NB_EPOCHS=1)")
    ap.add_argument("--shell", action="store_true", help="also run %%bash / ! cells")
    a = ap.parse_args(argv)
    env = dict(kv.split("=", 1) for kv in a.env)
    run_notebook(a.notebook, env=env, skip_shell=not a.shell)
    print("---- notebook finished: %s" % a.notebook)
    return 0


if __name__ == "__main__":
    sys.exit(main())
