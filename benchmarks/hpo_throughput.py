#!/usr/bin/env python
"""HPO throughput benchmark: RPV trials per hour on one MI355X node (BASELINE.json
"HPO trials/hour"; reference: 128 genetic-search evaluations of train_rpv -- 4 epochs,
64k train / 32k valid, batch 64 -- in 3h06m36s on 32 Cori nodes = 41.2 evals/hour,
``CrayHPO_rpv.ipynb:181,1282``).

Trials come from the DistHPO_rpv random-search space (``DistHPO_rpv.ipynb:91-106``),
each trains on one GPU (farm engine pinned per GPU), all GPUs busy concurrently.  The
synthetic dataset is generated once per engine and kept resident (device-side).  Wall
time covers farm start-up, every trial's model build / graph capture / training /
validation, and result collection.  Prints one JSON line.

``--mode cray`` measures the nested HPO x DP configuration instead (``CrayHPO_rpv.ipynb:
62-64,145-189``): an island-model genetic search whose every evaluation is a separate
``train_rpv`` process -- a ``torch.distributed.run`` data-parallel job of
``--gpus-per-eval`` ranks when that is > 1 -- scheduled over GPU slots by
``hpo.Evaluator``.  Wall time includes every evaluation's process start-up, which is what
the reference's 41.2 evaluations/hour paid too.  On a box with fewer GPUs than
``--gpus-per-eval`` the ranks of a slot share a GPU (gradients over gloo; said in the JSON).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REF_EVALS_PER_HOUR = 128 / (3 * 3600 + 6 * 60 + 36) * 3600     # 41.2
# flipped labels in every synthetic HPO data set: the tasks are not separable, so trials end
# at different val_loss above a ~H(0.1) floor and "best trial" is a real choice (the clean
# synthetic MNIST reached val_loss 1e-5 in round 3's driver run)
LABEL_NOISE = 0.1


def _cache():
    """Engine-resident dataset cache (trial functions are shipped by value, so a module
    global would be re-created for every task)."""
    from cori_intml_examples_amd.farm import engine_namespace
    return engine_namespace().setdefault("_hpo_bench_cache", {})


def trial(conv_sizes, fc_sizes, lr, dropout, optimizer, n_train=64000, n_valid=32000, batch_size=64,
          n_epochs=4, channels=1):
    import time as _t
    t0 = _t.time()
    from cori_intml_examples_amd.apps.rpv import build_model
    from cori_intml_examples_amd.io import synth
    model = build_model((64, 64, channels), conv_sizes=conv_sizes, fc_sizes=fc_sizes, dropout=dropout,
                        optimizer=optimizer, lr=lr)
    # the data set is generated ON the engine's GPU (K16 synth kernel) once and stays resident;
    # every trial's model shares its layout (same input shape)
    _CACHE = _cache()
    key = (n_train, n_valid, channels)
    if key not in _CACHE:
        _CACHE[key] = (synth.flip_labels(synth.for_model(model, "rpv", n_train, seed=1), LABEL_NOISE, 101),
                       synth.flip_labels(synth.for_model(model, "rpv", n_valid, seed=2), LABEL_NOISE, 102))
    tr, va = _CACHE[key]
    t1 = _t.time()
    h = model.fit(tr, None, batch_size=batch_size, epochs=n_epochs, validation_data=(va, None), verbose=0)
    return {"val_loss": h.history["val_loss"], "data_s": t1 - t0, "train_s": _t.time() - t1,
            "device": str(model.device), "t0": t0, "t1": _t.time()}


def trial_mnist(h1, h2, h3, dropout, optimizer, n_train=60000, batch_size=128, n_epochs=16, valid_frac=0.17):
    """DistHPO_mnist's build_and_train (DistHPO_mnist.ipynb:169-191) on cached synthetic MNIST."""
    import time as _t
    t0 = _t.time()
    from cori_intml_examples_amd.apps.mnist import build_model
    from cori_intml_examples_amd.io import synth
    model = build_model(h1=h1, h2=h2, h3=h3, dropout=dropout, optimizer=optimizer)
    _CACHE = _cache()
    key = ("mnist", n_train)
    if key not in _CACHE:      # generated on the engine's GPU (K16 synth kernel), resident
        _CACHE[key] = synth.flip_labels(synth.for_model(model, "mnist", n_train, seed=1), LABEL_NOISE, 103)
    data = _CACHE[key]
    t1 = _t.time()
    h = model.fit(data, None, batch_size=batch_size, epochs=n_epochs, validation_split=valid_frac, verbose=0)
    return {"val_loss": h.history["val_loss"], "data_s": t1 - t0, "train_s": _t.time() - t1,
            "device": str(model.device), "t0": t0, "t1": _t.time()}


def trial_rpv_widget(conv_sizes, fc_sizes, dropout, optimizer, lr, n_train=64000, n_valid=32000, batch_size=64,
                     n_epochs=2, channels=1):
    """DistWidgetHPO_rpv's build_and_train (``DistWidgetHPO_rpv.ipynb:160-168``): the RPV recipe
    (``apps.rpv.build_model`` / ``train_model``) with an ``IPyParallelLogger`` publishing
    every epoch to the dashboard, on cached synthetic RPV with label noise.  The logger also
    records when it published each message (same host clock as the polling client), so the
    driver can measure publish -> dashboard latency."""
    import time as _t
    t0 = _t.time()
    from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger
    from cori_intml_examples_amd.apps.rpv import build_model, train_model
    from cori_intml_examples_amd.io import synth

    class StampedLogger(IPyParallelLogger):
        def __init__(self):
            super().__init__()
            self.published = []          # (status, epoch, wall time)

        def _pub(self, status, epoch=None):
            super()._pub(status, epoch)
            self.published.append((status, epoch, _t.time()))

    model = build_model((64, 64, channels), conv_sizes=conv_sizes, fc_sizes=fc_sizes, dropout=dropout,
                        optimizer=optimizer, lr=lr)
    _CACHE = _cache()
    key = ("rpvw", n_train, n_valid, channels)
    if key not in _CACHE:
        _CACHE[key] = (synth.flip_labels(synth.for_model(model, "rpv", n_train, seed=1), LABEL_NOISE, 101),
                       synth.flip_labels(synth.for_model(model, "rpv", n_valid, seed=2), LABEL_NOISE, 102))
    tr, va = _CACHE[key]
    logger = StampedLogger()
    t1 = _t.time()
    h = train_model(model, tr, None, va, None, batch_size=batch_size, n_epochs=n_epochs, verbose=0,
                    callbacks=[logger])
    return {"val_loss": h.history["val_loss"], "data_s": t1 - t0, "train_s": _t.time() - t1,
            "published": logger.published, "device": str(model.device), "t0": t0, "t1": _t.time()}


def run_cray(a, n_gpu):
    """Genetic HPO whose evaluations are (DP) train_rpv processes; returns the JSON record."""
    import tempfile
    from cori_intml_examples_amd import hpo
    per = max(1, a.gpus_per_eval)
    if n_gpu >= per:
        slots = [list(range(i * per, (i + 1) * per)) for i in range(n_gpu // per)]
    elif n_gpu:
        slots = [[g % n_gpu for g in range(per)]]      # ranks share the GPU(s)
    else:
        slots = None
    params = hpo.Params([
        ["--h1", 16, (4, 64)], ["--h2", 32, (4, 64)], ["--h3", 64, (8, 128)], ["--h4", 128, (32, 256)],
        ["--dropout", 0.2, (0., 1.)], ["--optimizer", "Adam", ["Adam", "Nadam", "Adadelta"]],
        ["--lr", 1e-3, [1e-2, 1e-3, 1e-4]],
    ])
    cmd = ("python -m cori_intml_examples_amd.apps.train_rpv --synthetic --n-epochs %d --n-train %d "
           "--n-valid %d --batch-size %d --fom best --verbose 0" % (a.epochs, a.n_train, a.n_valid, a.batch_size))
    logd = tempfile.mkdtemp(prefix="cray-bench-")
    # verbose: one stderr line per finished evaluation (progress for long searches)
    ev = hpo.Evaluator(cmd, gpus_per_eval=per, slots=slots, slots_per_gpu=a.evals_per_slot,
                       timeout=a.eval_timeout, cpu_slots=2 if not n_gpu else None, cwd=ROOT,
                       env={"INTML_DEVICE": "cpu"} if not n_gpu else None, verbose=True)
    opt = hpo.GeneticOptimizer(ev, generations=a.generations, num_demes=a.demes, pop_size=a.pop_size,
                               log_fn=os.path.join(logd, "rpv_hpo.log"), seed=0)
    t0 = time.time()
    opt.optimize(params)
    wall = time.time() - t0
    hist = ev.history
    ok = [h for h in hist if h["ok"]]
    per_hour = len(ok) / wall * 3600
    # the data plane every evaluation's DP training reported (train_rpv's History.data_plane)
    planes = sorted({h.get("data_plane") or "none reported" for h in ok})
    return {
        "metric": "HPO evaluations/hour (CrayHPO_rpv genetic, %d-rank DP train_rpv per evaluation, %d epochs, "
                  "%d train / %d valid, batch %d/rank)" % (per, a.epochs, a.n_train, a.n_valid, a.batch_size),
        "value": round(per_hour, 1), "unit": "evaluations/hour", "n_gpus": n_gpu,
        "slots": len(ev.slots), "gpus_per_eval": per,
        "oversubscribed": any(ev.oversubscribed(sl) for sl in ev.slots),
        "data_plane": planes,
        "concurrent_evals": len(ev.slots),
        "evaluations": len(ok), "failed": len(hist) - len(ok), "wall_s": round(wall, 2),
        "mean_eval_s": round(sum(h["seconds"] for h in ok) / max(1, len(ok)), 2),
        "best_fom": min((h["fom"] for h in ok), default=None),
        "search": {"generations": a.generations, "demes": a.demes, "pop_size": a.pop_size},
        "vs_baseline": round(per_hour / REF_EVALS_PER_HOUR, 2),
        "baseline": "41.2 evals/hour (CrayHPO_rpv: 4-node DP evaluations, 32 Cori nodes)",
        "data": "synthetic RPV (1-channel 64x64), generated per evaluation process"}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--mode", choices=["farm", "cray"], default="farm",
                    help="farm: trials as farm tasks (DistHPO_*); cray: genetic search over DP train_rpv processes")
    ap.add_argument("--gpus-per-eval", type=int, default=1, help="cray mode: DP ranks per evaluation")
    ap.add_argument("--evals-per-slot", type=int, default=1, help="cray mode: concurrent evaluations per GPU slot")
    ap.add_argument("--generations", type=int, default=2)
    ap.add_argument("--demes", type=int, default=2)
    ap.add_argument("--pop-size", type=int, default=4)
    ap.add_argument("--eval-timeout", type=float, default=900.0)
    ap.add_argument("--trials", type=int, default=16)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--n-train", type=int, default=64000)
    ap.add_argument("--n-valid", type=int, default=32000)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--engines", type=int, default=None)
    ap.add_argument("--engines-per-gpu", type=int, default=4,
                    help="farm engines pinned to each GPU (small models leave most CUs idle)")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--model", choices=["rpv", "mnist"], default="rpv",
                    help="rpv: CrayHPO_rpv-style evaluations; mnist: DistHPO_mnist (16 epochs, 60k, B=128)")
    a = ap.parse_args(argv)
    argv_s = sys.argv if argv is None else list(argv)
    if a.model == "mnist":            # DistHPO_mnist.ipynb:137-153 defaults unless overridden
        a.epochs = a.epochs if "--epochs" in argv_s else 16
        a.n_train = a.n_train if "--n-train" in argv_s else 60000
        a.batch_size = a.batch_size if "--batch-size" in argv_s else 128
    import cloudpickle
    cloudpickle.register_pickle_by_value(sys.modules[__name__])
    from cori_intml_examples_amd import farm
    from cori_intml_examples_amd.hpo import random_search as rs
    n_gpu = 0 if a.cpu else farm.detect_gpus()
    if a.mode == "cray":
        rec = run_cray(a, n_gpu)
        print(json.dumps(rec), flush=True)
        return rec
    t0 = time.time()
    if a.engines is None:
        a.engines = max(1, n_gpu) * (a.engines_per_gpu if n_gpu else 1)
    cl = farm.start_cluster(a.engines, cluster_id="hpo_bench_%d" % os.getpid(),
                            cpu_only=a.cpu or n_gpu == 0, timeout=300)
    try:
        with cl.client() as c:
            t_up = time.time() - t0
            if a.model == "mnist":
                trials = rs.mnist_trials(a.trials)
                ars = rs.submit_trials(c.load_balanced_view(), trial_mnist, trials, n_train=a.n_train,
                                       batch_size=a.batch_size, n_epochs=a.epochs)
            else:
                trials = rs.rpv_trials(a.trials)
                ars = rs.submit_trials(c.load_balanced_view(), trial, trials, n_train=a.n_train, n_valid=a.n_valid,
                                       batch_size=a.batch_size, n_epochs=a.epochs)
            rs.wait_progress(ars, interval=1.0, printer=lambda s: print(s, file=sys.stderr, flush=True))
            res = rs.collect(ars)
    finally:
        cl.stop()
    wall = time.time() - t0
    ok = [r for r in res if r]
    per_hour = len(ok) / wall * 3600
    if a.model == "mnist":
        metric = ("HPO trials/hour (MNIST random search, %d epochs, %dk samples, valid_frac 0.17, batch %d)"
                  % (a.epochs, a.n_train // 1000, a.batch_size))
    else:
        metric = ("HPO trials/hour (RPV random search, %d epochs, %dk train / %dk valid, batch %d)"
                  % (a.epochs, a.n_train // 1000, a.n_valid // 1000, a.batch_size))
    rec = {
        "metric": metric,
        "value": round(per_hour, 1), "unit": "trials/hour", "n_gpus": n_gpu, "engines": a.engines,
        "trials": len(ok), "failed": len(res) - len(ok), "wall_s": round(wall, 2), "startup_s": round(t_up, 2),
        "mean_train_s": round(sum(r["train_s"] for r in ok) / max(1, len(ok)), 3),
        "mean_data_s": round(sum(r["data_s"] for r in ok) / max(1, len(ok)), 3),
        "mean_trial_s": round(sum(r["t1"] - r["t0"] for r in ok) / max(1, len(ok)), 3),
        # no like-for-like reference: CrayHPO_rpv's 41.2 evals/hour are 4-node DATA-PARALLEL
        # evaluations (batch 64/rank), these are single-GPU trials -- compare per evaluation
        # with --mode cray instead
        "vs_baseline": None,
        "baseline": ("not comparable: the reference's 41.2 evals/hour (CrayHPO_rpv) are 4-rank DP evaluations"
                     if a.model == "rpv" else "no wall-clock recorded"),
        "data": "synthetic %s, generated on each engine's GPU (K16 synth kernel), resident" % (
            "RPV (1-channel 64x64)" if a.model == "rpv" else "MNIST")}
    print(json.dumps(rec), flush=True)
    return rec


if __name__ == "__main__":
    main()
