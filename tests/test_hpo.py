"""HPO: golden random-search trial lists, Cray-style Params / Evaluator /
GeneticOptimizer with its log files (Appendix B.3), FoM protocol (B.5), sklearn grid
search wrapper, and a random search over CPU farm engines with live publish_data."""
import math
import os
import sys

import cloudpickle
import numpy as np
import pandas as pd
import pytest

from cori_intml_examples_amd import hpo
from cori_intml_examples_amd.hpo import random_search as rs

HERE = os.path.dirname(os.path.abspath(__file__))
FAKE = "python %s" % os.path.join(HERE, "helpers", "fom_quadratic.py")
cloudpickle.register_pickle_by_value(sys.modules[__name__])


def test_golden_trials():
    t = rs.mnist_trials(32)                           # DistHPO_mnist.ipynb:203,227
    assert rs.describe(t[0]) == "64-8-128 dropout 0.020 Nadam"
    assert rs.describe(t[24]) == "16-8-128 dropout 0.370 Adam"
    t = rs.mnist_trials(16)                           # HPO_mnist.ipynb:166-169
    assert (t[0]["h1"], t[0]["h2"], t[0]["h3"]) == (64, 8, 16) and round(t[0]["dropout"], 4) == 0.3865
    t = rs.mnist_trials(8)                            # DistWidgetHPO_mnist.ipynb best / worst
    assert rs.describe(t[4]) == "32-16-64 dropout 0.118 Adadelta"
    assert rs.describe(t[0]) == "64-64-16 dropout 0.979 Nadam"
    r = rs.rpv_trials(32)
    assert len(r[0]["conv_sizes"]) == 3 and len(r[0]["fc_sizes"]) == 1 and r[0]["lr"] in rs.RPV_LR


def test_best_trial_and_runtime():
    hs = [{"val_acc": [0.5, 0.9]}, None, {"val_acc": [0.95, 0.93]}, {"val_acc": [0.2, 0.97]}]
    assert rs.best_trial(hs) == (3, 0.97)
    assert rs.best_trial(hs, reduce="best") == (3, 0.97)
    assert rs.best_trial([{"val_loss": [0.3, 0.2]}, {"val_loss": [0.1, 0.4]}], "val_loss", "min", "best") == (1, 0.1)


def test_params_space():
    p = hpo.Params([["--h1", 16, (4, 64)], ["--dropout", 0.2, (0., 1.)], ["--optimizer", "Adam", ["Adam", "Nadam"]],
                    ["--lr", 1e-3, [1e-1, 1e-3, 1e-5]]])
    assert p.defaults() == {"--h1": 16, "--dropout": 0.2, "--optimizer": "Adam", "--lr": 1e-3}
    rng = np.random.RandomState(0)
    for _ in range(50):
        s = p.sample(rng)
        assert isinstance(s["--h1"], int) and 4 <= s["--h1"] <= 64
        assert 0.0 <= s["--dropout"] <= 1.0 and s["--optimizer"] in ("Adam", "Nadam")
        m = p.mutate(s, rng, 1.0)
        assert 4 <= m["--h1"] <= 64 and isinstance(m["--h1"], int)
    assert p.to_args(p.defaults()) == ["--h1", "16", "--dropout", "0.2", "--optimizer", "Adam", "--lr", "0.001"]
    with pytest.raises(ValueError):
        hpo.Params([["--a", 100, (0, 10)]])


def test_parse_fom():
    assert hpo.parse_fom("x\nFoM: 0.25\nmore") == 0.25
    assert hpo.parse_fom("FoM: 1e-3\nFoM: 2.5e-02") == 0.025
    assert hpo.parse_fom("no fom") is None


def test_evaluator_slots_and_failures(tmp_path):
    ev = hpo.Evaluator(FAKE, gpus=[], cpu_slots=3, log_dir=str(tmp_path / "logs"))
    foms = ev.evaluate([["--x", "0.3", "--n", "5", "--opt", "b"], ["--x", "0.99"], ["--x", "0.5", "--n", "5"]])
    assert foms[0] == pytest.approx(0.0) and math.isinf(foms[1]) and foms[2] == pytest.approx(0.54)
    assert len(os.listdir(tmp_path / "logs")) == 6
    # GPU-slot mapping: 8 "GPUs", 2 per evaluation -> 4 concurrent DP evaluations
    ev8 = hpo.Evaluator(FAKE, gpus=list(range(8)), gpus_per_eval=2)
    assert ev8.slots == [[0, 1], [2, 3], [4, 5], [6, 7]]
    cmd = ev8.command_for(["--x", "1"], [0, 1])
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node" in cmd


def test_evaluator_dp_launch():
    ev = hpo.Evaluator(FAKE, gpus=[], cpu_slots=1, nodes_per_eval=2, timeout=120)
    ev.per_eval = 2                        # CPU stand-in for a 2-GPU slot
    rec = ev.run_one(["--x", "0.3", "--n", "5", "--opt", "b"])
    assert rec["ok"] and rec["fom"] == pytest.approx(0.0), rec


def test_genetic_optimizer_logs(tmp_path):
    log = str(tmp_path / "hpo.log")
    params = hpo.Params([["--x", 0.8, (0.0, 1.0)], ["--n", 12, (0, 20)], ["--opt", "a", ["a", "b"]]])
    ev = hpo.Evaluator(FAKE, gpus=[], cpu_slots=4)
    opt = hpo.GeneticOptimizer(ev, generations=4, num_demes=2, pop_size=4, mutation_rate=0.5,
                               crossover_rate=0.33, log_fn=log, seed=1)
    best = opt.optimize(params)
    default_fom = (0.8 - 0.3) ** 2 + 49 / 100 + 0.5
    assert opt.best_fom < default_fom and set(best) == {"--x", "--n", "--opt"}
    summary = pd.read_csv(log, sep=r"\s+")
    assert list(summary.columns[:6]) == ["generation", "epoch", "best_fom", "avg_fom", "checkpoint_in",
                                         "checkpoint_out"]
    assert list(summary.generation) == [0, 1, 2, 3] and summary.best_fom.is_monotonic_decreasing
    demes = [pd.read_csv(str(tmp_path / ("Deme%d_hpo.log" % d)), sep=r"\s+") for d in (1, 2)]
    allr = pd.concat(demes, ignore_index=True)
    assert len(allr) == 4 * 2 * 4 and list(allr.columns[:4]) == ["generation", "tag", "fitness", "FoM"]
    assert allr.fitness.between(0, 1).all() and allr.tag.iloc[0] == "deme1_ind0"
    assert allr.iloc[0]["--x"] == 0.8                 # generation 0 starts from the defaults
    assert hpo.genetic.Optimizer is hpo.GeneticOptimizer


def _build_small(h1=4, h2=4, h3=8, dropout=0.0):
    from cori_intml_examples_amd.apps.zoo import mnist_cnn
    return mnist_cnn(h1=h1, h2=h2, h3=h3, dropout=dropout, input_shape=(12, 12, 1), device="cpu")


def test_sklearn_grid_search():
    from sklearn.model_selection import GridSearchCV
    from cori_intml_examples_amd.io.datasets import synthetic_mnist
    x, y, _, _ = synthetic_mnist(240, 10, rows=12, cols=12)
    sk = hpo.KerasClassifier(build_fn=_build_small, batch_size=32, epochs=2, verbose=0)
    grid = GridSearchCV(sk, dict(h1=[4, 8], dropout=[0.0]), cv=2)
    grid.fit(x, y)
    res = pd.DataFrame(grid.cv_results_)
    assert len(res) == 2 and res.mean_test_score.between(0, 1).all()
    assert grid.best_estimator_.predict(x[:5]).shape == (5,)
    assert grid.best_estimator_.predict_proba(x[:5]).shape == (5, 10)


def _build_and_train(h1, h2, h3, dropout, optimizer, n_epochs=1):
    from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger, configure_session
    from cori_intml_examples_amd.apps.zoo import mnist_cnn
    from cori_intml_examples_amd.io.datasets import synthetic_mnist
    configure_session()
    x, y, _, _ = synthetic_mnist(300, 10, rows=12, cols=12)
    m = mnist_cnn(h1=h1, h2=h2, h3=h3, dropout=dropout, optimizer=optimizer, input_shape=(12, 12, 1))
    h = m.fit(x, y, batch_size=64, epochs=n_epochs, validation_split=0.17, verbose=2,
              callbacks=[IPyParallelLogger()])
    return h.history


def test_random_search_on_farm():
    from cori_intml_examples_amd import farm
    cl = farm.start_cluster(2, cluster_id="pytest_hpo_%d" % os.getpid(), cpu_only=True, timeout=120)
    try:
        with cl.client() as c:
            trials = [dict(t, h1=4, h2=4, h3=8) for t in rs.mnist_trials(3)]
            ars = rs.submit_trials(c.load_balanced_view(), _build_and_train, trials, n_epochs=2)
            rs.wait_progress(ars, interval=0.2, timeout=300, printer=lambda s: None)
            hs = rs.collect(ars)
            assert all(h is not None and len(h["val_acc"]) == 2 for h in hs)
            assert ars[0].data["status"] == "Ended Training"
            assert ars[0].data["history"]["epoch"] == [0, 1]
            assert "Train on 249 samples, validate on 51 samples" in ars[0].stdout
            i, v = rs.best_trial(hs)
            assert 0 <= i < 3 and 0 <= v <= 1
            assert (rs.runtime_seconds(ars) > 0).all()
    finally:
        cl.stop()


def test_evaluator_timeout_kills_whole_process_group(tmp_path):
    """A timed-out evaluation takes its children with it (a torchrun launcher cannot
    forward SIGKILL to its ranks): no grandchild survives the timeout."""
    import signal
    import time
    from cori_intml_examples_amd.hpo.evaluator import run_group
    pidfile = tmp_path / "child.pid"
    script = ("import subprocess, sys, time\n"
              "p = subprocess.Popen([sys.executable, '-c', 'import signal, time; "
              "signal.signal(signal.SIGTERM, signal.SIG_IGN); time.sleep(600)'])\n"
              "open(%r, 'w').write(str(p.pid))\n"
              "time.sleep(600)\n" % str(pidfile))
    t0 = time.time()
    out, err, rc = run_group([sys.executable, "-c", script], timeout=3, grace=1.0)
    assert rc == -9 and "timeout" in err and time.time() - t0 < 30
    pid = int(pidfile.read_text())
    for _ in range(50):            # the SIGKILLed grandchild is reaped by init shortly
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            break
        with open("/proc/%d/stat" % pid) as f:
            if f.read().split()[2] == "Z":
                break
        time.sleep(0.1)
    else:
        os.kill(pid, signal.SIGKILL)
        raise AssertionError("grandchild %d survived the evaluation timeout" % pid)


def test_evaluator_explicit_and_shared_gpu_slots(monkeypatch):
    """Explicit slots; a slot naming one GPU twice runs 2 ranks on it (they select the RCCL-free
    xGMI data plane themselves: more local ranks than visible GPUs -- no gloo override);
    slots_per_gpu repeats slots (several evaluations per GPU) -- and then the GPU's concurrent
    multi-rank evaluations use gloo (the xGMI plane bounds its spinning workgroups
    per job, not across jobs)."""
    monkeypatch.delenv("INTML_DP_BACKEND", raising=False)
    monkeypatch.delenv("INTML_COMM", raising=False)
    one = hpo.Evaluator("python -c pass", gpus_per_eval=2, slots=[[0, 0]])
    env = one._env_for([0, 0])
    assert env["HIP_VISIBLE_DEVICES"] == "0" and "INTML_DP_BACKEND" not in env and "INTML_COMM" not in env
    ev = hpo.Evaluator("python -c pass", gpus_per_eval=2, slots=[[0, 0]], slots_per_gpu=3)
    assert ev.num_slots == 3 and ev.gpus == [0]
    assert ev.oversubscribed([0, 0]) and not ev.oversubscribed([0, 1])
    assert ev.shared_across_slots([0, 0]) and not one.shared_across_slots([0, 0])
    env = ev._env_for([0, 0])
    assert env["HIP_VISIBLE_DEVICES"] == "0" and env["INTML_DP_BACKEND"] == "gloo" and env["INTML_COMM"] == "torch"
    two = hpo.Evaluator("python -c pass", gpus_per_eval=2, slots=[[0, 1], [1, 2]])   # overlapping slots
    assert two._env_for([0, 1])["INTML_DP_BACKEND"] == "gloo"
    env = hpo.Evaluator("python -c pass", gpus_per_eval=2, slots=[[2, 3]])._env_for([2, 3])
    assert env["HIP_VISIBLE_DEVICES"] == "2,3" and "INTML_DP_BACKEND" not in env
    cmd = ev.command_for(["--lr", "0.1"], [0, 0])
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "2" in cmd
    with pytest.raises(ValueError):
        hpo.Evaluator("python -c pass", gpus_per_eval=2, slots=[[0]])


def test_cray_bench_cpu():
    """bench.py --hpo cray: genetic search over 2-rank DP train_rpv processes (gloo on CPU)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--hpo", "cray", "--", "--cpu",
                        "--generations", "1", "--demes", "1", "--pop-size", "2", "--n-train", "256",
                        "--n-valid", "128", "--epochs", "1"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["unit"] == "evaluations/hour" and rec["evaluations"] == 2 and rec["failed"] == 0
    assert rec["gpus_per_eval"] == 2 and rec["value"] > 0


def test_figure_of_merit_nan_safe():
    """FoM ("best" = min val_loss, "last") never lets a NaN epoch win and scores an all-NaN
    (diverged) trial NaN, which the genetic optimizer ranks worst; min() with a NaN in the
    list would be order-dependent."""
    import math
    from cori_intml_examples_amd.hpo.evaluator import figure_of_merit, parse_fom
    nan = float("nan")
    assert figure_of_merit([0.5, 0.3, 0.4]) == 0.3
    assert figure_of_merit([nan, 0.3]) == 0.3 and figure_of_merit([0.3, nan]) == 0.3
    assert math.isnan(figure_of_merit([nan, nan])) and math.isnan(figure_of_merit([]))
    assert figure_of_merit([0.2, 0.4], "last") == 0.4
    assert math.isnan(figure_of_merit([0.2, float("inf")], "last"))
    assert math.isnan(parse_fom("FoM: nan"))
    from cori_intml_examples_amd.hpo.genetic import _fitness
    f = _fitness([0.5, nan, 0.2])
    assert f[1] == min(f) and f[2] == max(f)
