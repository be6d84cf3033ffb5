"""Evaluator: runs a training command per hyper-parameter point and parses its figure of
merit (``hpo.Evaluator``, ``CrayHPO_rpv.ipynb:145-151``; FoM protocol ``train_rpv.py:
76-79``).

The reference's evaluator allocated SLURM nodes (``nodes``, ``nodes_per_eval``,
``alloc_args``, ``launcher='wlm'``) and ran each evaluation as a multi-node Horovod job.
On one MI355X node the unit is the GPU: the ``gpus`` of the node are cut into slots of
``gpus_per_eval`` (alias ``nodes_per_eval``) and each evaluation runs on one slot --
``HIP_VISIBLE_DEVICES`` pinned, and, when a slot has more than one GPU, launched as a
data-parallel job (``torch.distributed.run``, one rank per GPU, its own RCCL communicator
on 127.0.0.1:<own port>) -- nested HPO x DP.  Slots run concurrently.

``slots`` gives the slot list explicitly instead (one list of GPU ids per slot).  A slot
that names one GPU more than once runs that many ranks on it (oversubscription: a 1-GPU
box can still run a 2-rank nested evaluation); RCCL needs distinct devices per rank, so
such a slot's ranks select the RCCL-free xGMI data plane on their own (``dist.init``: more
local ranks than visible GPUs) -- the same fused all-reduce + optimizer kernel over
IPC-mapped peer memory that a multi-GPU job uses, captured into the step graph.
``slots_per_gpu`` > 1 repeats every slot that many times (several small evaluations share a
GPU concurrently, as the farm's engines-per-GPU do); multi-rank evaluations on a GPU shared by
concurrent slots use the gloo data plane (``_env_for``: the xGMI plane's spinning workgroups
are bounded per job, not across jobs).

An evaluation whose command fails or prints no ``FoM:`` line scores ``inf`` (worst);
``retries`` re-runs it first.  Each run's stdout/stderr goes to ``log_dir`` if given.
"""
from __future__ import annotations

import os
import queue
import math
import re
import shlex
import socket
import subprocess
import sys
import threading
import time
from typing import Any, Dict, List, Optional, Sequence

# the gradient data plane an evaluation's training ran on (train_rpv prints History.data_plane)
_PLANE = re.compile(r"gradient reducer ([^\n]+)")
_FOM = re.compile(r"FoM:\s*([-+]?(?:\d+\.?\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|inf|nan))")


def parse_fom(text: str) -> Optional[float]:
    """Last ``FoM: <float>`` in ``text`` (every DP rank prints it; they agree)."""
    m = _FOM.findall(text or "")
    return float(m[-1]) if m else None


def figure_of_merit(val_losses: Sequence[float], mode: str = "best") -> float:
    """The FoM a training CLI prints (``train_rpv.py:76-79``): the min ("best") or last
    validation loss.  Non-finite epochs (a diverged trial's NaN/inf losses) never win the
    min -- Python's ``min`` with a NaN in the list is order-dependent -- and a run with no
    finite epoch (or a non-finite last epoch in "last" mode) scores NaN, which the
    evaluators and the genetic optimizer rank worst."""
    vals = [float(v) for v in val_losses]
    if not vals:
        return float("nan")
    if mode == "last":
        return vals[-1] if math.isfinite(vals[-1]) else float("nan")
    fin = [v for v in vals if math.isfinite(v)]
    return min(fin) if fin else float("nan")


def run_group(cmd: Sequence[str], env=None, timeout: Optional[float] = None, cwd=None,
              grace: float = 10.0):
    """Run ``cmd`` in its OWN session / process group; returns (stdout, stderr, rc).

    On timeout the whole group gets SIGTERM, then SIGKILL after ``grace`` seconds: a
    ``torch.distributed.run`` launcher cannot forward a SIGKILL to its worker ranks, which
    would otherwise stay alive holding the slot's GPUs, RCCL communicators and port."""
    import signal
    p = subprocess.Popen(cmd, env=env, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
        return out, err, p.returncode
    except subprocess.TimeoutExpired:
        pgid = p.pid           # start_new_session: the child leads its own group

        def _kill(sig):
            try:
                os.killpg(pgid, sig)
            except ProcessLookupError:
                pass
        _kill(signal.SIGTERM)
        try:
            out, _ = p.communicate(timeout=grace)    # EOF only once every group member is gone
        except subprocess.TimeoutExpired:
            _kill(signal.SIGKILL)
            out, _ = p.communicate()
        _kill(signal.SIGKILL)      # a straggler that closed its pipes but ignored SIGTERM
        return out or "", "timeout after %ss" % timeout, -9


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Evaluator:
    def __init__(self, cmd: str, nodes: Optional[int] = None, nodes_per_eval: int = 1,
                 alloc_args: Optional[str] = None, launcher: str = "local", verbose: bool = False,
                 gpus: Optional[Sequence[int]] = None, gpus_per_eval: Optional[int] = None,
                 timeout: Optional[float] = None, env: Optional[Dict[str, str]] = None, retries: int = 0,
                 log_dir: Optional[str] = None, cwd: Optional[str] = None, cpu_slots: Optional[int] = None,
                 slots: Optional[Sequence[Sequence[int]]] = None, slots_per_gpu: int = 1):
        self.cmd = cmd
        self.per_eval = int(gpus_per_eval or nodes_per_eval or 1)
        if gpus is None:
            from ..farm.cluster import detect_gpus
            n = detect_gpus()
            if nodes is not None and n:
                n = min(n, int(nodes))
            gpus = list(range(n))
        self.gpus = list(gpus)
        self.alloc_args, self.launcher, self.verbose = alloc_args, launcher, verbose
        self.timeout, self.retries, self.log_dir, self.cwd = timeout, int(retries), log_dir, cwd
        self.env = dict(env or {})
        if slots is not None:
            self.slots = [list(sl) for sl in slots]
            if any(len(sl) != self.per_eval for sl in self.slots):
                raise ValueError("every slot must list gpus_per_eval=%d GPU ids" % self.per_eval)
            self.gpus = sorted({g for sl in self.slots for g in sl})
        elif self.gpus:
            if len(self.gpus) < self.per_eval:
                raise ValueError("gpus_per_eval=%d but only %d GPUs" % (self.per_eval, len(self.gpus)))
            self.slots = [self.gpus[i * self.per_eval:(i + 1) * self.per_eval]
                          for i in range(len(self.gpus) // self.per_eval)]
        else:       # no GPU on this host: CPU slots (tests, dry runs)
            n = cpu_slots or (int(nodes) // self.per_eval if nodes else 2)
            self.slots = [None] * max(1, n)
        if slots_per_gpu > 1:
            self.slots = [sl for sl in self.slots for _ in range(int(slots_per_gpu))]
        self.history: List[Dict[str, Any]] = []
        self._lock = threading.Lock()
        self._count = 0
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)

    def shared_across_slots(self, slot) -> bool:
        """True if a GPU of ``slot`` also belongs to another slot (evaluations that run
        concurrently on one GPU)."""
        if slot is None:
            return False
        mine = set(slot)
        return sum(1 for sl in self.slots if sl is not None and mine & set(sl)) > 1

    @property
    def num_slots(self) -> int:
        return len(self.slots)

    def command_for(self, args: Sequence[str], slot, rank_log_dir: Optional[str] = None) -> List[str]:
        base = shlex.split(self.cmd)
        if base and os.path.basename(base[0]).startswith("python"):
            base = [sys.executable] + base[1:]
        if self.per_eval > 1:
            rest = base[1:] if base and base[0] == sys.executable else base
            base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                    str(self.per_eval), "--master-addr", "127.0.0.1", "--master-port", str(_free_port())]
            if rank_log_dir:      # per-rank stdout files: concurrent ranks cannot interleave the FoM line
                base += ["--log-dir", rank_log_dir, "--redirects", "3"]
            # "--": the script's own flags (e.g. --n) must not be prefix-matched by torchrun
            if rest[:1] == ["-m"]:
                base += ["-m", "--"] + rest[1:]
            else:
                base += ["--"] + rest
        return base + list(args)

    @staticmethod
    def _rank_output(log_dir: str, rank: int = 0) -> str:
        for d, _, files in os.walk(log_dir):
            if os.path.basename(d) == str(rank) and "stdout.log" in files:
                with open(os.path.join(d, "stdout.log")) as f:
                    return f.read()
        return ""

    def _env_for(self, slot) -> Dict[str, str]:
        env = dict(os.environ)
        env.update(self.env)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if slot is not None:
            uniq = list(dict.fromkeys(slot))
            env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in uniq)
            # (ranks sharing a GPU -- LOCAL_RANK % visible devices -- take the RCCL-free xGMI
            # plane: dist.init sees more local ranks than devices.)  A GPU that several
            # CONCURRENT evaluations share (slots_per_gpu > 1, or overlapping slots) is
            # different: each job caps its spinning all-reduce workgroups from its own ranks
            # only, so jobs could starve each other's launches of CUs -- their
            # multi-rank evaluations keep the gloo data plane, which does not spin on the GPU
            if self.per_eval > 1 and self.shared_across_slots(slot):
                env["INTML_COMM"] = "torch"
                env["INTML_DP_BACKEND"] = "gloo"
        else:
            env.setdefault("INTML_DEVICE", "cpu")
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        return env

    def run_one(self, args: Sequence[str], slot=None, tag: str = "") -> Dict[str, Any]:
        rec: Dict[str, Any] = {"args": list(args), "slot": slot, "tag": tag}
        import tempfile
        for attempt in range(self.retries + 1):
            tmp = tempfile.mkdtemp(prefix="intml-eval-") if self.per_eval > 1 else None
            cmd = self.command_for(args, slot, tmp)
            t0 = time.time()
            out, err, rc = run_group(cmd, env=self._env_for(slot), timeout=self.timeout, cwd=self.cwd)
            if tmp is not None:
                import shutil
                out = self._rank_output(tmp, 0) + out
                shutil.rmtree(tmp, ignore_errors=True)
            fom = parse_fom(out) if rc == 0 else None
            plane = _PLANE.search(out)
            rec.update(cmd=cmd, rc=rc, seconds=time.time() - t0, attempt=attempt,
                       fom=float("inf") if fom is None else fom, ok=fom is not None,
                       data_plane=plane.group(1).strip() if plane else None)
            if self.log_dir:
                with self._lock:
                    self._count += 1
                    n = self._count
                base = os.path.join(self.log_dir, "eval%04d%s" % (n, ("_" + tag) if tag else ""))
                with open(base + ".out", "w") as f:
                    f.write(" ".join(cmd) + "\n" + out)
                with open(base + ".err", "w") as f:
                    f.write(err)
            else:
                rec["stdout_tail"] = out[-2000:]
                rec["stderr_tail"] = err[-2000:]
            if rec["ok"]:
                break
        if self.verbose:
            print("[eval %s] %s -> FoM %s (%.1fs%s)" % (tag or "-", " ".join(args), rec["fom"], rec["seconds"],
                                                      "" if rec["ok"] else ", FAILED rc=%s" % rec["rc"]),
                  flush=True)
        with self._lock:
            self.history.append(rec)
        return rec

    def evaluate(self, points: Sequence[Sequence[str]], tags: Optional[Sequence[str]] = None) -> List[float]:
        """Run every argument list (concurrently over the slots); FoMs in input order."""
        tags = list(tags) if tags is not None else [""] * len(points)
        results: List[Optional[Dict[str, Any]]] = [None] * len(points)
        work: "queue.Queue" = queue.Queue()
        for i, p in enumerate(points):
            work.put(i)

        def worker(slot):
            while True:
                try:
                    i = work.get_nowait()
                except queue.Empty:
                    return
                results[i] = self.run_one(points[i], slot, tags[i])

        threads = [threading.Thread(target=worker, args=(s,), daemon=True) for s in self.slots]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        return [r["fom"] for r in results]

    @staticmethod
    def oversubscribed(slot) -> bool:
        return slot is not None and len(set(slot)) < len(slot)

    def __repr__(self):
        return "Evaluator(%r, slots=%d x %d GPU)" % (self.cmd, self.num_slots, self.per_eval)
