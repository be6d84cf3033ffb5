"""Data parallelism with 2 gloo ranks on the CPU (the multi-process path the driver runs
with RCCL on 8 MI355X): collectives, state broadcast, DP step == single-process step on
the global batch, lockstep training, and the ``train_rpv`` CLI under torchrun."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(nproc, args, timeout=300):
    env = dict(os.environ)
    env.update({"INTML_DEVICE": "cpu", "PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2"})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)


def test_dp_invariants(tmp_path):
    r = _torchrun(2, [os.path.join(ROOT, "tests", "dp_worker.py"), str(tmp_path)])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    reps = [json.load(open(tmp_path / ("rank%d.json" % i))) for i in range(2)]
    for rep in reps:
        assert rep["size"] == 2
        assert rep["allreduce_sum"] == 3.0 and rep["allreduce_avg"] == 1.5
        assert rep["allgather"] == [0, 10]
        assert rep["broadcast"] == [1.0] * 4
        assert rep["broadcast_object"] == {"from": 0}
        assert rep["history_keys"] == ["acc", "loss", "lr", "val_acc", "val_loss"]
    assert reps[1]["init_differs"] > 0            # seeds differed before the broadcast
    assert reps[0]["w1_digest"] == reps[1]["w1_digest"]
    assert reps[0]["dp_vs_single_maxdiff"] < 1e-5
    assert reps[0]["wf_digest"] == reps[1]["wf_digest"]
    # MetricAverageCallback: every rank reports the same (averaged) epoch metrics
    assert reps[0]["val_loss"] == reps[1]["val_loss"]
    assert reps[0]["loss"] == reps[1]["loss"]


def test_train_rpv_cli_two_ranks(tmp_path):
    logs = str(tmp_path / "logs")
    r = _torchrun(2, ["--log-dir", logs, "--redirects", "3", "-m", "cori_intml_examples_amd.apps.train_rpv", "--n-train", "256", "--n-valid", "64",
                      "--n-epochs", "1", "--batch-size", "32", "--fom", "best", "--lr-scaling", "linear",
                      "--input-dir", "/nonexistent", "--h1", "4", "--h2", "8", "--h3", "8", "--h4", "16"])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    outs = []
    for rank in range(2):
        found = [os.path.join(d, "stdout.log") for d, _, fs in os.walk(logs)
                 if "stdout.log" in fs and os.path.basename(d) == str(rank)]
        assert found, os.listdir(logs)
        outs.append(open(found[0]).read())
    foms = [[l for l in o.splitlines() if l.startswith("FoM:")] for o in outs]
    assert len(foms[0]) == 1 and foms[0] == foms[1]     # weights + averaged metrics agree
    assert "MPI rank 0" in outs[0] and "MPI rank 1" in outs[1]
    assert "Total params" in outs[0] and "Total params" not in outs[1]   # rank-0 summary only
