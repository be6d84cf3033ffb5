"""bench.py's data-plane probe (N > 1): picks the fastest eligible plane, sets its env for the
timed run, rejects a plane whose probe left the ranks' weights different, and stays out of
the way when INTML_XGMI / INTML_BUCKET_BYTES pin the plane.  CPU, with the model build,
the timing and the collectives stubbed (the real path needs >= 2 GPUs)."""
import os
import sys
import types

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cori_intml_examples_amd.parallel import hvd  # noqa: E402


@pytest.fixture
def probe_env(monkeypatch):
    monkeypatch.setenv("INTML_PLANE_VERDICTS", "/nonexistent-dir/verdicts.json")   # (unwritable: no file)
    for k in ("INTML_XGMI", "INTML_BUCKET_BYTES", "INTML_PLANE_PROBE"):
        # setenv first so teardown restores the original state even though the probe itself
        # writes these variables
        monkeypatch.setenv(k, "")
        monkeypatch.delenv(k)
    cost = {"xgmi": 10.0, "rccl": 11.0, "rccl_forked": 12.0, "hybrid": 13.0}
    sums = {"bad": set()}

    def plane():
        if os.environ.get("INTML_XGMI") in ("xgmi", "hybrid"):
            return os.environ["INTML_XGMI"]
        return "rccl_forked" if os.environ.get("INTML_BUCKET_BYTES") else "rccl"

    def build(args, size, dp, dev):
        x = (types.SimpleNamespace(err=[types.SimpleNamespace(item=lambda: 0)]) if plane() in ("xgmi", "hybrid")
             else None)
        m = types.SimpleNamespace(_executor=types.SimpleNamespace(reducer=types.SimpleNamespace(xgmi=x)),
                                  plane=plane(), store=types.SimpleNamespace(numel=547841))
        return m, (64, 64, 3), 1, "cfg", "metric", None

    monkeypatch.setattr(bench, "build", build)
    monkeypatch.setattr(bench, "synthetic", lambda *a, **k: None)
    monkeypatch.setattr(bench, "time_steps", lambda m, *a, **k: (cost[m.plane] * 1e-3, [1.0]))
    monkeypatch.setattr(bench, "weight_checksum", lambda m: [1.0, 2.0, 3.0])
    monkeypatch.setattr(hvd, "broadcast_global_variables", lambda *a, **k: None)

    def allgather(v):   # two ranks; rank 1's weights differ for the planes marked bad
        if isinstance(v, list) and len(v) == 2 and isinstance(v[0], list):
            other = [[9.0, 2.0, 3.0], True] if plane() in sums["bad"] else v
            return [v, other]
        return [v, v]

    monkeypatch.setattr(hvd, "allgather", allgather)
    args = types.SimpleNamespace(via_fit=False, samples=1024, warmup=30)
    return cost, sums, args


def test_probe_picks_fastest_and_sets_env(probe_env):
    cost, _, args = probe_env
    cost.update(xgmi=12.0, rccl=11.0, rccl_forked=10.0)
    r = bench.probe_data_planes(args, 2, None, None, 128, 8)
    assert r["chosen"] == "rccl_forked" and set(r) >= {"xgmi", "rccl", "rccl_forked", "hybrid"}
    assert os.environ["INTML_XGMI"] == "rccl" and os.environ["INTML_BUCKET_BYTES"] == str(1 << 20)


def test_probe_records_verdict(probe_env, monkeypatch, tmp_path):
    """The probe's choice is persisted (rank 0) for fit()'s auto plane: the plane family under
    the job's (host, world size, gradient size class) key."""
    import json
    from cori_intml_examples_amd.parallel import dist as D
    cost, _, args = probe_env
    monkeypatch.setenv("INTML_PLANE_VERDICTS", str(tmp_path / "v.json"))
    cost.update(xgmi=9.0)
    r = bench.probe_data_planes(args, 2, None, None, 128, 8)
    assert r["chosen"] == "xgmi" and r["verdict_file"] == str(tmp_path / "v.json")
    d = json.load(open(tmp_path / "v.json"))
    (k, v), = d.items()
    assert k == D.verdict_key(2, 4 * 547841) and v["plane"] == "xgmi" and v["probe_ms_per_step"]["xgmi"] > 0


def test_probe_can_pick_hybrid(probe_env):
    cost, _, args = probe_env
    cost.update(xgmi=12.0, rccl=11.0, rccl_forked=10.5, hybrid=9.0)
    r = bench.probe_data_planes(args, 2, None, None, 128, 8)
    assert r["chosen"] == "hybrid"
    assert os.environ["INTML_XGMI"] == "hybrid" and os.environ["INTML_BUCKET_BYTES"] == str(1 << 20)


def test_default_plane_is_rccl(monkeypatch, tmp_path):
    """Without a probe verdict (fit(), train_rpv) the data plane is RCCL: nothing but a
    measurement admits xGMI (the verdict path is tests/test_comm.py::
    test_auto_plane)."""
    from cori_intml_examples_amd.parallel.dist import data_plane
    monkeypatch.delenv("INTML_XGMI", raising=False)
    monkeypatch.setenv("INTML_PLANE_VERDICTS", str(tmp_path / "none.json"))
    assert data_plane() == "rccl" and data_plane(4 * 547841) == "rccl"
    for v, want in (("auto", "rccl"), ("0", "rccl"), ("1", "xgmi"), ("xgmi", "xgmi"), ("hybrid", "hybrid")):
        monkeypatch.setenv("INTML_XGMI", v)
        assert data_plane() == want


def test_probe_rejects_divergent_plane(probe_env):
    cost, sums, args = probe_env
    sums["bad"].add("xgmi")                    # fastest, but its ranks ended with different weights
    r = bench.probe_data_planes(args, 2, None, None, 128, 8)
    assert r["xgmi"] is None and "xgmi_rejected" in r and r["chosen"] == "rccl"
    assert os.environ["INTML_XGMI"] == "rccl" and "INTML_BUCKET_BYTES" not in os.environ


def test_probe_respects_pinned_plane(probe_env, monkeypatch):
    _, _, args = probe_env
    monkeypatch.setenv("INTML_XGMI", "1")
    assert bench.probe_data_planes(args, 2, None, None, 128, 8) is None
    assert bench.probe_data_planes(args, 1, None, None, 128, 8) is None


def test_inline_hpo_record_on_cpu(monkeypatch):
    """bench.py's inline HPO (the 'hpo' record of the JSON line): the farm starts before the
    training bench, runs the DistHPO_mnist trials after it and reports trials/hour.  CPU
    engines and a shrunken search here; the GPU run uses 64 trials x 16 epochs x 60k."""
    from cori_intml_examples_amd import farm
    monkeypatch.setattr(farm, "detect_gpus", lambda: 0)
    monkeypatch.setattr(bench.InlineHpo, "TRIALS", 3)
    monkeypatch.setattr(bench.InlineHpo, "EPOCHS", 1)
    monkeypatch.setattr(bench.InlineHpo, "SAMPLES", 600)
    # DistWidgetHPO_rpv record: 3 concurrent trials (8 on the GPU), tiny data
    monkeypatch.setattr(bench.InlineHpo, "RPV_TRIALS", 3)
    monkeypatch.setattr(bench.InlineHpo, "RPV_TRAIN", 256)
    monkeypatch.setattr(bench.InlineHpo, "RPV_VALID", 128)
    h = bench.InlineHpo(engines_per_gpu=2, budget_s=120.0, rpv_budget_s=240.0)
    try:
        recs = h.run()
    finally:
        h.stop()
    assert h.engines == 2 and h.rpv_engines == 3   # the search's farm; the RPV record's own farm
    rec = recs["hpo"]
    assert rec["trials_done"] == 3 and not rec["capped"], rec
    assert rec["trials_per_hour"] > 0 and rec["wall_s"] >= rec["startup_s"] > 0
    assert rec["epochs"] == 1 and rec["samples"] == 600 and rec["engines_per_gpu"] == 2
    assert rec["label_noise"] == 0.1
    rr = recs["hpo_rpv"]
    assert rr["trials_done"] == 3 and not rr["capped"] and rr["concurrent"] == 3, rr
    # every trial's epochs reached the dashboard model (2 epochs each) and were timed
    assert rr["dashboard_rows_final"] == [2, 2, 2], rr
    assert rr["epoch_messages_seen"] == 6 and rr["publish_to_dashboard_ms_p50"] is not None, rr
    assert rr["publish_to_dashboard_ms_p50"] >= 0 and rr["best_val_loss"] > 0, rr
