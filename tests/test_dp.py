"""Data parallelism with 2 gloo ranks on the CPU (the multi-process path the driver runs
with RCCL on 8 MI355X): collectives, state broadcast, DP step == single-process step on
the global batch, lockstep training, and the ``train_rpv`` CLI under torchrun."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(nproc, args, timeout=300, extra_env=None):
    env = dict(os.environ)
    env.update({"INTML_DEVICE": "cpu", "PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1" if nproc > 2 else "2"})
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_dp_invariants(tmp_path, n):
    """n gloo ranks (the driver runs the same path with RCCL on 2/4/8 MI355X); a 256-byte
    bucket cap splits the gradient into many backward-ordered buckets."""
    r = _torchrun(n, [os.path.join(ROOT, "tests", "dp_worker.py"), str(tmp_path)],
                  extra_env={"INTML_BUCKET_BYTES": "256"}, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    reps = [json.load(open(tmp_path / ("rank%d.json" % i))) for i in range(n)]
    tri = n * (n + 1) / 2
    for rep in reps:
        assert rep["size"] == n
        assert rep["allreduce_sum"] == tri and rep["allreduce_avg"] == tri / n
        assert rep["allgather"] == [10 * i for i in range(n)]
        assert rep["broadcast"] == [1.0] * 4
        assert rep["broadcast_object"] == {"from": 0}
        assert rep["history_keys"] == ["acc", "loss", "lr", "val_acc", "val_loss"]
        # buckets: backward order (descending offsets), disjoint, covering [0, numel) exactly
        b = rep["buckets"]
        assert len(b) > 2
        assert all(b[i][0] == b[i + 1][1] for i in range(len(b) - 1))
        assert b[0][1] == rep["numel"] and b[-1][0] == 0
        assert b == reps[0]["buckets"]
    assert all(rep["init_differs"] > 0 for rep in reps[1:])     # seeds differed before the broadcast
    for rep in reps[1:]:
        assert rep["w1_digest"] == reps[0]["w1_digest"]
        assert rep["wf_digest"] == reps[0]["wf_digest"]
        # MetricAverageCallback: every rank reports the same (averaged) epoch metrics
        assert rep["val_loss"] == reps[0]["val_loss"]
        assert rep["loss"] == reps[0]["loss"]
    assert reps[0]["dp_vs_single_maxdiff"] < 1e-5


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
    assert "rank 0/2" in outs[0] and "rank 1/2" in outs[1]
    assert "Total params" in outs[0] and "Total params" not in outs[1]   # rank-0 summary only


def test_shard_indices_disjoint_cover_and_reshard():
    """Distributed sampler of fit(): per epoch the ranks' slices are disjoint, equal-sized,
    drawn from one permutation; shards change across epochs (the n % size left-outs too)."""
    from cori_intml_examples_amd.train.loop import shard_indices
    n, size = 1003, 4
    seen_left_out = set()
    prev = None
    for epoch in range(3):
        parts = [shard_indices(n, r, size, True, 12345, epoch) for r in range(size)]
        assert all(len(p) == n // size for p in parts)
        allidx = np.concatenate([p.numpy() for p in parts])
        assert len(set(allidx.tolist())) == len(allidx)            # disjoint
        assert allidx.min() >= 0 and allidx.max() < n
        left = set(range(n)) - set(allidx.tolist())
        assert len(left) == n % size
        seen_left_out |= left
        if prev is not None:
            assert not np.array_equal(prev, parts[0].numpy())     # reshuffled shard
        prev = parts[0].numpy()
    assert len(seen_left_out) > n % size                             # not the same samples forever
    # same seed + epoch -> the same slices on every rank (no communication needed per epoch)
    assert np.array_equal(shard_indices(n, 2, size, True, 7, 5).numpy(), shard_indices(n, 2, size, True, 7, 5).numpy())
    # unshuffled: the contiguous fixed-shard layout
    assert np.array_equal(shard_indices(10, 1, 3, False, 0, 0).numpy(), np.arange(3, 6))


@pytest.mark.parametrize("scenario", ["all_init", "one_init", "uid", "hang", "late", "selftest", "ok"])
def test_rccl_failure_falls_back_collectively(tmp_path, scenario):
    """A multi-GPU job whose RCCL data plane fails to come up -- in any phase (unique id,
    communicator construction, a rank that never joins, the numeric self-test), on every rank
    or on ONE rank only -- moves EVERY rank onto the RCCL-free xGMI data plane through the
    phased votes of comm.establish: no rank raises, no rank hangs (2 ranks, gloo, CPU)."""
    r = _torchrun(2, [os.path.join(ROOT, "tests", "comm_fallback_worker.py"), str(tmp_path), scenario],
                  timeout=120, extra_env={"INTML_RCCL_INIT_TIMEOUT": "4"})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    reps = [json.load(open(tmp_path / ("fb%d.json" % i))) for i in range(2)]
    assert all(rep["size"] == 2 for rep in reps), reps
    if scenario == "ok":
        assert all(rep["comm"] and not rep["xgmi_only"] and rep["plane"].startswith("rccl") for rep in reps), reps
        return
    assert all(rep["xgmi_only"] and not rep["comm"] and rep["plane"].startswith("xgmi") for rep in reps), reps
    if scenario in ("one_init", "hang", "selftest"):
        assert reps[0]["aborted"] == 1, reps        # rank 0's healthy communicator was aborted
    if scenario == "hang":
        assert all(rep["init_s"] < 60 for rep in reps), reps
    if scenario == "late":
        # rank 1's communicator came up after the deadline: the reaper aborted and closed it
        # (no live communicator + watchdog left behind on the RCCL-free plane)
        assert reps[1]["abandoned"] == ["closed"] and reps[1]["aborted"] == 1 and reps[1]["closed"] == 1, reps
        assert reps[0]["abandoned"] == [] and reps[0]["aborted"] == 1, reps


@pytest.mark.parametrize("scenario", ["ok", "diverge"])
def test_fit_detects_divergent_rank(tmp_path, scenario):
    """fit()'s per-epoch cross-rank weight digest: identical ranks record one
    identical digest per epoch; a rank that diverged (injected on rank 1 at epoch 1) makes
    fit() raise DataParallelDivergence on EVERY rank at that epoch's end, with the failing
    record in History.dp_consistency (2 gloo ranks)."""
    r = _torchrun(2, [os.path.join(ROOT, "tests", "dp_diverge_worker.py"), str(tmp_path), scenario], timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    reps = [json.load(open(tmp_path / ("div%d.json" % i))) for i in range(2)]
    if scenario == "ok":
        for rep in reps:
            assert rep["raised"] is None and rep["epochs_done"] == 3, rep
            assert [x["epoch"] for x in rep["records"]] == [0, 1, 2] and all(x["identical"] for x in rep["records"])
        assert reps[0]["records"] == reps[1]["records"]
        return
    for rep in reps:
        assert rep["raised"] and "epoch 1" in rep["raised"] and "[1]" in rep["raised"], rep
        assert [x["identical"] for x in rep["records"]] == [True, False], rep
        assert rep["records"][-1]["ranks_differing"] == [1]


@pytest.mark.parametrize("scenario", ["rank0", "rank1"])
def test_plane_choice_is_rank0s(tmp_path, scenario):
    """One data plane per job (2 gloo ranks): only one rank sees an xGMI verdict for the job's
    key; NativeGradReducer.configure broadcasts rank 0's choice, so both ranks run xGMI when
    rank 0 has the verdict and both stay on RCCL when only rank 1 does."""
    r = _torchrun(2, [os.path.join(ROOT, "tests", "plane_vote_worker.py"), str(tmp_path), scenario], timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    reps = [json.load(open(tmp_path / ("vote%d.json" % i))) for i in range(2)]
    holder = 1 if scenario == "rank1" else 0
    assert reps[holder]["local_view"] == "xgmi" and reps[1 - holder]["local_view"] == "rccl", reps
    want = "xgmi" if holder == 0 else "rccl"
    assert [x["plane"] for x in reps] == [want, want], reps
