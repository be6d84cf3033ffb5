#!/usr/bin/env python
"""Headline benchmark: RPV CNN training throughput (images/sec, whole job).

BASELINE.json metric "images/sec (whole node) RPV CNN at 1/2/4/8 MI355X"; config
"ATLAS RPV 3-channel calorimeter-image CNN data-parallel bf16 (DistTrain_rpv)":
conv [16,32,64] 3x3 'same' + ReLU + 2x2 max-pool, Dropout(0.2), Dense(128)+ReLU,
Dropout(0.2), Dense(1)+sigmoid, binary cross-entropy, Adam(lr = 0.001 * size),
batch 128 per rank (DistTrain_rpv.ipynb:267-285), 64x64x3 input.

Each timed step is a FULL training step: device-side batch gather from the resident
(synthetic) dataset by the epoch permutation, forward, loss, backward, bucketed RCCL
gradient all-reduce (N > 1) with each bucket's Adam update behind it, weight re-pack.
Weak scaling: per-GPU batch fixed.  Launch: ``python bench.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.

Self-check at N > 1 (the multi-GPU path is never run by the builder; the run proves
itself): the line reports the rank count the RCCL communicator reports, the gradient
bucket sizes, per-rank step-time p50/max, a cross-rank checksum of the trained weights
and the exposed communication time (the same step without DP, same N, timed right after);
the process exits with status 3 if the checksums differ or RCCL saw the wrong rank count.
Before the timed run, unless ``INTML_XGMI`` / ``INTML_BUCKET_BYTES`` pin it, a short probe
times the full DP step on each data plane (fused xGMI kernel, one RCCL all-reduce, forked
RCCL buckets overlapping the backward) and the fastest is timed (``probe_data_planes``; the
probe numbers and the choice are in the self-check).

``--via-fit`` times what users run instead: ``apps.rpv.train_model(...)`` epochs
(Keras fit loop, Horovod callbacks, optional ``--lr-warmup-epochs``), training images only.

HPO trials/hour (BASELINE.json's second metric) rides on the same JSON line as ``"hpo"``:
rank 0 starts a task farm on every visible GPU BEFORE anything touches the GPU (engines are
child processes; nothing is forked from a GPU-initialised process), the training bench runs
and is timed while the engines idle, the data-parallel group shuts down, and then the farm
runs the DistHPO_mnist random search (``DistHPO_mnist.ipynb:137-255``: 64 trials, 16 epochs,
60k samples, valid_frac 0.17, batch 128, load-balanced over the engines), capped at
``--hpo-budget`` seconds including engine start-up (a capped run reports the trials it
finished), and then BASELINE config 5 as ``"hpo_rpv"``: DistWidgetHPO_rpv's 8 concurrent RPV
trials monitored live by the dashboard model (``InlineHpo``).  ``--no-hpo`` skips both.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
BASELINE_LEGACY_IMG_PER_S = 1240.0   # RPV legacy CNN (34.5M params), 1 GPU, Train_rpv.ipynb:304-312
BASELINE_MNIST_IMG_PER_S = 43600.0   # MNIST DP aggregate, 8 Haswell nodes, DistTrain_mnist.ipynb:341-357


@contextlib.contextmanager
def _quiet_stdout():
    """fit() banners / callback prints go to stderr: stdout carries ONE JSON line."""
    old = sys.stdout
    sys.stdout = sys.stderr
    try:
        yield
    finally:
        sys.stdout = old


def build(args, size, dp, dev):
    from cori_intml_examples_amd.apps import zoo
    if args.model == "rpv":
        model = zoo.rpv_cnn((64, 64, args.channels), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2,
                            optimizer="Adam", lr=0.001 * size, use_horovod=dp, device=dev)
        shape, ncls = (64, 64, args.channels), 1
        cfg = "RPV CNN conv[16,32,64] fc[128] 64x64x%d (DistTrain_rpv)" % args.channels
        # no reference throughput exists for this 547,841-param model (the
        # DistTrain_rpv training cell's timing was not saved) -> vs_baseline null
        metric, baseline = "images/sec (whole node) RPV CNN training", None
    elif args.model == "mnist":
        model = zoo.mnist_cnn(32, 64, 128, 0.25, 0.5, lr=1.0 * size, use_horovod=dp, device=dev)
        shape, ncls = (28, 28, 1), 10
        cfg = "MNIST CNN 32-64-128 (DistTrain_mnist)"
        metric, baseline = "images/sec (whole node) MNIST CNN training", BASELINE_MNIST_IMG_PER_S
    else:
        model = zoo.rpv_legacy_cnn((64, 64, args.channels), device=dev, use_horovod=dp)
        shape, ncls = (64, 64, args.channels), 1
        cfg = "RPV legacy CNN 34.5M (Train_rpv)"
        metric, baseline = "images/sec (whole node) RPV legacy CNN training", BASELINE_LEGACY_IMG_PER_S
    return model, shape, ncls, cfg, metric, baseline


def synthetic(n, shape, ncls, ex, dev, g):
    """The bench's data set, generated on the device by the K16 synth kernel (io/synth.py):
    RPV-like jet images (binary heads) or MNIST-like class templates (10 classes), in the
    executor's layout, resident for the whole run."""
    import torch
    from cori_intml_examples_amd.io import synth
    seed = int(torch.randint(0, 1 << 31, (1,), generator=g, device=dev).item())
    return synth.synth_device("rpv" if ncls == 1 else "mnist", n, shape, ncls, ex.in_Cs, seed, dev)


def time_steps(model, data, B, steps, warmup, chunk, g, dev, settle_ms=0.0, info=None):
    """Warmup (captures every graph the timed loop replays), then time `steps` full training
    steps as graph replays of `chunk` steps.  Returns (elapsed seconds on this rank, per-step
    ms of each replay from HIP events).

    settle_ms > 0: before the timed region, replay the timed graph back to back (no host sync
    between replays) until the GPU has run it for ~settle_ms.  The chip's power management
    holds a lower clock until it has been under sustained load for ~10-15 ms; the driver's
    short command (--steps 20 --warmup 5: ~3 ms of work before its timed region) otherwise
    times the ramp, not the step -- every kernel of the step runs 3-5 % slower in it and an
    idle gap of 200 ms puts it back (profiles/r5_driver_gap.txt).  The settle steps are
    reported on the JSON line (``settle_steps`` / ``settle_ms``), never folded into ``warmup``."""
    import torch
    from cori_intml_examples_amd.parallel import hvd
    ex = model._executor
    n = data.n
    state = {"pos": 0, "perm": torch.randperm(n, device=dev, generator=g)}

    def run(k):
        if state["pos"] + k * B > n:
            state["pos"] = 0
            state["perm"] = torch.randperm(n, device=dev, generator=g)
        ex.train_steps(data, state["perm"], state["pos"], B, k)
        state["pos"] += k * B

    def chunks(total):
        return [chunk] * (total // chunk) + ([total % chunk] if total % chunk else [])

    ex.reset_metrics()
    timed = chunks(steps)
    for k in chunks(warmup) + sorted(set(timed)):
        run(k)
    if settle_ms > 0 and timed:
        k = max(timed)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(k)
        e1.record()
        torch.cuda.synchronize()
        reps = max(1, int(-(-settle_ms // max(e0.elapsed_time(e1), 1e-3))))
        t0 = time.perf_counter()
        for _ in range(reps):
            run(k)
        torch.cuda.synchronize()
        if info is not None:
            info["settle_steps"] = (reps + 1) * k
            info["settle_ms"] = round((time.perf_counter() - t0) * 1e3 + e0.elapsed_time(e1), 2)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(timed) + 1)]
    hvd.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    for i, k in enumerate(timed):
        run(k)
        evs[i + 1].record()
    torch.cuda.synchronize()
    hvd.barrier()
    t1 = time.perf_counter()
    per_step = [evs[i].elapsed_time(evs[i + 1]) / k for i, k in enumerate(timed)]
    return t1 - t0, per_step


def weight_checksum(model):
    import torch
    m = model.store.master[:model.store.numel].double()
    return [float(m.sum()), float(m.abs().sum()), float((m * m).sum())]


def probe_data_planes(args, size, dev, g, B, chunk):
    """Data-plane autotune at N > 1 (the Horovod-autotune analogue for the choice that matters
    here; SURVEY.md §5.1 item 3 "benchmark it against RCCL and keep the winner"): unless
    ``INTML_XGMI`` / ``INTML_BUCKET_BYTES`` pin it, time a short probe of the full DP step on
    each candidate data plane --
      xgmi         the xGMI plane (fit()'s default on one node, dist.auto_plane): the head /
                   dense range pushed to its owners, all-reduced and updated inside the
                   backward (exchange), the conv layers' in the end-of-backward reduction,
      xgmi_end     the xGMI plane with the exchange as a launch of its own after the backward,
      rccl         the RCCL plane: one all-reduce + optimizer of the whole gradient at the end
                   of the backward (dist.adaptive_bucket_bytes),
      rccl_single  one RCCL all-reduce of the whole gradient at the end of the backward,
      rccl_forked  1 MiB buckets in backward order, each all-reduce forked onto the comm
                   stream as soon as its gradients are reduced (overlaps the conv backward),
      hybrid       the dense bucket's RCCL all-reduce forked onto the comm stream (overlaps the
                   conv backward) + the small conv bucket through the fused xGMI kernel,
    MAX over ranks, and keep the fastest for the timed run (its env is set, so every later
    build agrees).  Every probe is complete training steps; the choice is collective (the same
    numbers on every rank).  Returns {plane: ms/step}, or None if there was nothing to choose."""
    from cori_intml_examples_amd.parallel import hvd
    forced = os.environ.get("INTML_PLANE_PROBE", "0") == "1"     # also at N = 1 (loopback test)
    if ((size < 2 and not forced) or args.via_fit or "INTML_XGMI" in os.environ
            or "INTML_BUCKET_BYTES" in os.environ):
        return None
    base_tune = os.environ.get("INTML_TUNE", "")
    end_tune = ",".join(x for x in (base_tune, "xchg_at=end") if x)
    cands = (("xgmi", {"INTML_XGMI": "xgmi"}),
             # the exchange as its own launch after the backward: 2 us less fixed cost, the early
             # range's all-reduce no longer overlapping the conv backward -- the wire decides
             ("xgmi_end", {"INTML_XGMI": "xgmi", "INTML_TUNE": end_tune}),
             ("rccl", {"INTML_XGMI": "rccl"}),
             ("rccl_single", {"INTML_XGMI": "rccl", "INTML_BUCKET_BYTES": str(1 << 40)}),
             ("rccl_forked", {"INTML_XGMI": "rccl", "INTML_BUCKET_BYTES": str(1 << 20)}),
             ("hybrid", {"INTML_XGMI": "hybrid", "INTML_BUCKET_BYTES": str(1 << 20)}))
    probe = max(chunk * 6, 48)
    res = {}
    numel = None
    for plane, env in cands:
        os.environ.update(env)
        try:
            model, shape, ncls, *_ = build(args, size, True, dev)
            numel = model.store.numel
            hvd.broadcast_global_variables(0, model=model)
            data = synthetic(max(args.samples, B * 4), shape, ncls, model._executor, dev, g)
            e, _ = time_steps(model, data, B, probe, min(args.warmup, 16), chunk, g, dev,
                              settle_ms=min(getattr(args, "settle_ms", 0.0), 20.0))
            # the reducer sets the xGMI plane up at its first step (collective self-test + vote)
            x = getattr(model._executor.reducer, "xgmi", None)
            on = plane not in ("xgmi", "hybrid") or x is not None
            # a plane is only eligible if it trained correctly here: no timed-out wait and
            # bit-identical weights on every rank after the probe steps
            sane = [weight_checksum(model), bool(x is None or int(x.err[0].item()) == 0)]
            sane = hvd.allgather(sane) if size > 1 else [sane]
            ok = all(c == sane[0][0] and f for c, f in sane)
            res[plane] = (round((max(hvd.allgather(e)) if size > 1 else e) / probe * 1e3, 4)
                          if on and ok else None)
            if not ok:
                res[plane + "_rejected"] = "weights differ across ranks or a wait timed out"
            del model, data
        except Exception as e:        # noqa: BLE001 -- a plane that cannot run is not chosen
            res[plane] = None
            res[plane + "_rejected"] = ("%s: %s" % (type(e).__name__, e))[:200]
        finally:
            for k in env:
                os.environ.pop(k, None)
            if base_tune:
                os.environ["INTML_TUNE"] = base_tune
    best = min(((v, k) for k, v in res.items() if isinstance(v, float)), default=(0, "rccl"))[1]
    os.environ.update(dict(cands)[best])
    res["chosen"] = best
    # persist the measured choice for fit()'s auto plane on this host / world size / gradient
    # size class (dist.auto_plane: without a verdict, auto means RCCL)
    if numel and any(isinstance(v, float) for v in res.values()) and (not hvd.is_initialized() or hvd.rank() == 0):
        from cori_intml_examples_amd.parallel import dist as D
        res["verdict_file"] = D.record_verdict(size, 4 * numel, best,
                                               {k: v for k, v in res.items() if isinstance(v, float)})
    return res


def run_fit(args, model, shape, ncls, size, dp):
    """Time `apps.rpv.train_model` epochs (the recipe path: Keras fit loop + Horovod
    callbacks); the first epoch (graph capture) is untimed."""
    import numpy as np
    import torch
    from cori_intml_examples_amd.apps.rpv import train_model
    from cori_intml_examples_amd.train import callbacks as cbks
    rs = np.random.RandomState(1234)
    n = max(args.samples // 2, args.batch * 8) // args.batch * args.batch
    x = rs.rand(n, *shape).astype(np.float32)
    y = (rs.rand(n) > 0.5).astype(np.float32) if ncls == 1 else rs.randint(0, ncls, n)
    marks = []

    class EpochClock(cbks.Callback):
        needs_batch_logs = False

        def on_epoch_begin(self, epoch, logs=None):
            torch.cuda.synchronize()
            marks.append([time.perf_counter(), None])

        def on_epoch_end(self, epoch, logs=None):
            torch.cuda.synchronize()       # (the loop already synced reading the epoch metrics)
            marks[-1][1] = time.perf_counter()

    epochs = max(2, args.fit_epochs)
    with _quiet_stdout():
        train_model(model, x, y, None, None, batch_size=args.batch, n_epochs=epochs,
                    lr_warmup_epochs=args.lr_warmup_epochs, use_horovod=dp, verbose=0,
                    callbacks=[EpochClock()])
    per_rank = n // size if (dp and size > 1) else n      # fit() shards the data set per rank
    timed = marks[1:]
    elapsed = sum(b - a for a, b in timed)
    steps = len(timed) * (per_rank // args.batch)
    return elapsed, steps, [(b - a) / (per_rank // args.batch) * 1e3 for a, b in timed]


def run_hpo(args, extra):
    """HPO trials/hour on the BASELINE configs (benchmarks/hpo_throughput.py; one JSON line).
    Runs in this process before anything touches the GPU (the farm engines / evaluation
    processes own the GPUs)."""
    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    import hpo_throughput
    extra = [e for e in extra if e != "--"]
    if args.hpo == "mnist":     # BASELINE: 64 MNIST trials (DistHPO_mnist: 16 epochs, 60k, B=128)
        argv = ["--model", "mnist", "--trials", "64"]
    elif args.hpo == "rpv":     # BASELINE config 5: RPV CNN, 8 concurrent trials (DistWidgetHPO_rpv)
        argv = ["--model", "rpv", "--trials", "8", "--engines-per-gpu", "8"]
    else:                       # CrayHPO_rpv: nested HPO x DP, 2-rank evaluations
        argv = ["--mode", "cray", "--gpus-per-eval", "2", "--generations", "2", "--demes", "2", "--pop-size", "4"]
    hpo_throughput.main(argv + extra)
    return 0


class InlineHpo:
    """The HPO records of the JSON line, on ONE task farm started before the training bench
    touches the GPU and used after it (see the module docstring):

    * ``hpo``      DistHPO_mnist random search: 64 trials (16 epochs, 60k, valid_frac 0.17,
                   B=128) load-balanced over ``engines_per_gpu`` engines of every GPU;
    * ``hpo_rpv``  DistWidgetHPO_rpv (BASELINE config 5): 8 CONCURRENT RPV trials of the
                   notebook's search space (``DistWidgetHPO_rpv.ipynb:113-125``: conv / fc /
                   lr / dropout / optimizer, B=64, 2 epochs, 64k train / 32k valid) through
                   ``apps.rpv.train_model`` with an ``IPyParallelLogger`` each, monitored live
                   by the headless dashboard model (``widgets.ParamSpanModel.poll``, the
                   ParamSpanWidget's update loop) -- trials/hour plus the publish -> dashboard
                   latency of the epoch messages.
    Both data sets carry 10 % flipped labels (benchmarks/hpo_throughput.LABEL_NOISE)."""

    TRIALS, EPOCHS, SAMPLES, BATCH, VALID_FRAC = 64, 16, 60000, 128, 0.17
    RPV_TRIALS, RPV_EPOCHS, RPV_TRAIN, RPV_VALID, RPV_BATCH = 8, 2, 64000, 32000, 64

    def __init__(self, engines_per_gpu: int, budget_s: float, rpv_budget_s: float = 60.0):
        from cori_intml_examples_amd import farm
        self.t0 = time.time()
        self.budget_s = budget_s
        self.rpv_budget_s = rpv_budget_s
        self.n_gpu = farm.detect_gpus()
        g = max(1, self.n_gpu)
        # the MNIST search's farm: engines_per_gpu engines of every GPU.  The RPV record's 8
        # concurrent engines are a farm of their own, started after the search: starting
        # them together with the search's (8 engine processes initialising at once on the
        # box's CPU share) doubled the search's wall time (4.2k trials/h against 7.7-8.3k)
        self.epg = engines_per_gpu
        self.engines = g * self.epg
        self.rpv_engines = g * -(-self.RPV_TRIALS // g)
        self.cl = farm.start_cluster(self.engines, cluster_id="bench_hpo_%d" % os.getpid(),
                                     cpu_only=self.n_gpu == 0, timeout=min(120.0, budget_s))
        self.startup_s = time.time() - self.t0
        self.cl_rpv = None

    def run(self):
        from cori_intml_examples_amd import farm
        out = {}
        try:
            with self.cl.client() as c:
                out["hpo"] = self._mnist(c)
        finally:
            self.cl.stop()
        try:
            t = time.time()
            self.cl_rpv = farm.start_cluster(self.rpv_engines, cluster_id="bench_hpo_rpv_%d" % os.getpid(),
                                             cpu_only=self.n_gpu == 0, timeout=min(120.0, self.rpv_budget_s))
            startup = time.time() - t
            with self.cl_rpv.client() as c:
                out["hpo_rpv"] = self._rpv(c, startup)
        except Exception as e:     # noqa: BLE001 -- the MNIST record must survive
            out["hpo_rpv"] = {"error": str(e)[:300]}
        finally:
            if self.cl_rpv is not None:
                self.cl_rpv.stop()
        return out

    def _mnist(self, c):
        import cloudpickle
        sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
        import hpo_throughput
        from cori_intml_examples_amd.hpo import random_search as rs
        cloudpickle.register_pickle_by_value(hpo_throughput)
        t1 = time.time()
        g = max(1, self.n_gpu)
        view = c.load_balanced_view()           # the search's own farm: every engine
        trials = rs.mnist_trials(self.TRIALS)
        ars = rs.submit_trials(view, hpo_throughput.trial_mnist, trials, n_train=self.SAMPLES,
                               batch_size=self.BATCH, n_epochs=self.EPOCHS, valid_frac=self.VALID_FRAC)
        deadline = t1 + max(1.0, self.budget_s - self.startup_s)
        while not all(a.ready() for a in ars) and time.time() < deadline:
            time.sleep(0.25)
        t2 = time.time()
        capped = not all(a.ready() for a in ars)
        done = [r for r in rs.collect([a for a in ars if a.ready()]) if r]
        for a in ars:
            if not a.ready():
                a.abort()
        wall = self.startup_s + (t2 - t1)
        best = min((min(r["val_loss"]) for r in done), default=None)
        return {"metric": "HPO trials/hour (DistHPO_mnist random search)",
                "trials_per_hour": round(len(done) / wall * 3600, 1), "trials_done": len(done),
                "trials_submitted": self.TRIALS, "capped": capped, "n_gpus": self.n_gpu,
                "engines_per_gpu": self.epg, "epochs": self.EPOCHS,
                "samples": self.SAMPLES, "valid_frac": self.VALID_FRAC, "batch": self.BATCH,
                "wall_s": round(wall, 2), "startup_s": round(self.startup_s, 2), "search_s": round(t2 - t1, 2),
                "mean_trial_s": round(sum(r["t1"] - r["t0"] for r in done) / max(1, len(done)), 3),
                "best_val_loss": best, "budget_s": self.budget_s,
                "label_noise": hpo_throughput.LABEL_NOISE,
                "data": "synthetic MNIST (60k, 10% flipped labels) generated on each engine GPU by the K16 "
                        "kernel, resident; random-init weights"}

    def _rpv(self, c, startup_s: float):
        import functools
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
        import hpo_throughput
        from cori_intml_examples_amd.hpo import random_search as rs
        from cori_intml_examples_amd.widgets.model import ModelController, ParamSpanModel
        trials = rs.rpv_trials(self.RPV_TRIALS)            # DistWidgetHPO_rpv.ipynb:113-125, seed 0
        params = {k: [t[k] for t in trials] for k in ("conv_sizes", "fc_sizes", "dropout", "optimizer", "lr")}
        fn = functools.partial(hpo_throughput.trial_rpv_widget, n_train=self.RPV_TRAIN, n_valid=self.RPV_VALID,
                               batch_size=self.RPV_BATCH, n_epochs=self.RPV_EPOCHS)
        ctl = ModelController(client=c, view=c.load_balanced_view())   # its own farm: 8 engines
        psm = ParamSpanModel(fn, params, controller=ctl)
        seen = {}                                           # (row, epoch) -> first time on the dashboard

        def on_change(what, i):
            if what == "row":
                now = time.time()
                for e in range(psm.data[i].num_data_rows):
                    seen.setdefault((i, e), now)

        psm.listeners.append(on_change)
        t1 = time.time()
        psm.submit_computations(poll=False)
        deadline = t1 + self.rpv_budget_s
        polls = 0
        while time.time() < deadline:
            psm.poll()
            polls += 1
            if not ctl.get_running_models():
                break
            time.sleep(0.02)
        t2 = time.time()
        futs = psm.results
        capped = not all(f is not None and f.ready() for f in futs)
        done = []
        for f in futs:
            if f is not None and f.ready():
                try:
                    done.append(f.get())
                except Exception:   # noqa: BLE001
                    pass
            elif f is not None:
                f.abort()
        lat = []
        for i, f in enumerate(futs):
            if f is None or not f.ready():
                continue
            try:
                r = f.get()
            except Exception:       # noqa: BLE001
                continue
            for status, epoch, tp in r["published"]:
                if status == "Ended Epoch" and (i, epoch) in seen:
                    lat.append(seen[(i, epoch)] - tp)
        # one convention for both HPO records: wall_s includes the farm start-up (reported on
        # its own as startup_s too), trials/hour = trials / wall_s
        wall = startup_s + (t2 - t1)
        best = min((min(r["val_loss"]) for r in done), default=None)
        return {"metric": "HPO trials/hour (DistWidgetHPO_rpv: %d concurrent RPV trials, live dashboard)"
                          % self.RPV_TRIALS,
                "trials_per_hour": round(len(done) / wall * 3600, 1), "trials_done": len(done),
                "trials_submitted": self.RPV_TRIALS, "capped": capped, "n_gpus": self.n_gpu,
                "engines_per_gpu": -(-self.RPV_TRIALS // max(1, self.n_gpu)), "concurrent": self.RPV_TRIALS,
                "epochs": self.RPV_EPOCHS, "n_train": self.RPV_TRAIN, "n_valid": self.RPV_VALID,
                "batch": self.RPV_BATCH, "wall_s": round(wall, 2), "startup_s": round(startup_s, 2),
                "search_s": round(t2 - t1, 2),
                "mean_trial_s": round(sum(r["t1"] - r["t0"] for r in done) / max(1, len(done)), 3),
                "best_val_loss": best, "dashboard_polls": polls,
                "publish_to_dashboard_ms_p50": round(float(np.median(lat)) * 1e3, 2) if lat else None,
                "publish_to_dashboard_ms_max": round(float(np.max(lat)) * 1e3, 2) if lat else None,
                "epoch_messages_seen": len(lat),
                "dashboard_rows_final": [int(psm.data[i].num_data_rows) for i in range(psm.n_models)],
                "label_noise": hpo_throughput.LABEL_NOISE,
                "data": "synthetic RPV (1-channel 64x64, 10% flipped labels) generated on each engine GPU by the "
                        "K16 kernel, resident; random-init weights"}

    def stop(self):
        for cl in (self.cl, self.cl_rpv):
            try:
                if cl is not None:
                    cl.stop()
            except Exception:     # noqa: BLE001
                pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=128, help="per-GPU batch (reference: 128)")
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--samples", type=int, default=32768, help="resident synthetic samples per rank")
    ap.add_argument("--model", default="rpv", choices=["rpv", "mnist", "rpv_legacy"])
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--steps-per-graph", type=int, default=int(os.environ.get("INTML_STEPS_PER_GRAPH", 32)),
                    help="full training steps per HIP-graph replay (32: +0.7 %% over 8, profiles/r4q_spg.txt; "
                         "fit() replays INTML_STEPS_PER_GRAPH, default 8, between its callbacks)")
    ap.add_argument("--settle-ms", type=float, default=60.0,
                    help="before the timed steps, replay the timed graph back to back for ~this long so the "
                         "GPU clock has left its power-management ramp (reported as settle_steps / settle_ms; "
                         "0 = off; profiles/r5_driver_gap.txt)")
    ap.add_argument("--no-dp-delta", action="store_true",
                    help="skip the DP-off re-run that measures the exposed communication time")
    ap.add_argument("--via-fit", action="store_true", help="time apps.rpv.train_model epochs (Keras fit path)")
    ap.add_argument("--fit-epochs", type=int, default=4)
    ap.add_argument("--lr-warmup-epochs", type=int, default=0)
    ap.add_argument("--hpo", choices=["mnist", "rpv", "cray"], default=None,
                    help="instead of the training-step bench, measure HPO throughput (BASELINE.json's "
                         "second metric): mnist = 64 DistHPO_mnist trials spread over the node's GPUs, "
                         "rpv = DistWidgetHPO_rpv-style 8 concurrent RPV trials, cray = genetic search over "
                         "2-rank DP train_rpv evaluations; extra flags after -- go to benchmarks/hpo_throughput.py")
    ap.add_argument("--no-hpo", action="store_true",
                    help="skip the DistHPO_mnist trials/hour measurement reported as 'hpo' on the JSON line")
    ap.add_argument("--hpo-budget", type=float, default=90.0, help="seconds for the inline HPO, start-up included")
    ap.add_argument("--hpo-engines-per-gpu", type=int, default=4)
    args, extra = ap.parse_known_args()
    if args.hpo:
        return run_hpo(args, extra)
    if extra:
        ap.error("unrecognized arguments: %s" % " ".join(extra))
    if args.no_graphs:
        os.environ["INTML_GRAPHS"] = "0"
    # rank 0 starts the HPO farm now, before this process initialises the GPU
    inline_hpo = None
    if not args.no_hpo and not args.via_fit and int(os.environ.get("RANK", "0")) == 0:
        try:
            inline_hpo = InlineHpo(args.hpo_engines_per_gpu, args.hpo_budget)
            import atexit
            atexit.register(inline_hpo.stop)      # no engine outlives a failed bench
        except Exception as e:   # noqa: BLE001 -- the training metric must not depend on it
            print("inline HPO farm failed to start: %s" % e, file=sys.stderr, flush=True)

    import torch
    from cori_intml_examples_amd.parallel import hvd

    st = hvd.init()
    rank, size = hvd.rank(), hvd.size()
    local = hvd.local_rank()
    torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
    dev = torch.device("cuda", torch.cuda.current_device())
    os.environ.setdefault("INTML_DEVICE", str(dev))

    B = args.batch
    # INTML_DP_FORCE=1 runs the full data-parallel step (RCCL all-reduces in the graph) at N=1
    dp = size > 1 or os.environ.get("INTML_DP_FORCE", "0") not in ("0", "")
    chunk = max(1, args.steps_per_graph)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    plane_probe = probe_data_planes(args, size, dev, g, B, chunk) if dp else None
    model, shape, ncls, cfg_name, metric, baseline = build(args, size, dp, dev)
    ex = model._executor

    if args.via_fit:
        elapsed, steps, per_step = run_fit(args, model, shape, ncls, size, dp)
        warmup_note = "1 epoch (untimed)"
    else:
        data = synthetic(max(args.samples, B * 4), shape, ncls, ex, dev, g)
        hvd.broadcast_global_variables(0, model=model)
        settle = {}
        elapsed, per_step = time_steps(model, data, B, args.steps, args.warmup, chunk, g, dev,
                                       settle_ms=args.settle_ms, info=settle)
        steps = args.steps
        warmup_note = args.warmup
    loss = ex.read_metrics()[0]

    # ---------------------------------------------------------------- self-check (DP)
    selfcheck, ok = None, True
    stats = {"p50": sorted(per_step)[len(per_step) // 2], "max": max(per_step)}
    if size > 1:
        elapsed = max(hvd.allgather(elapsed))   # MAX over ranks
        steps = min(hvd.allgather(steps))
    if dp:
        comm = st.comm
        red = ex.reducer
        sums = hvd.allgather(weight_checksum(model)) if size > 1 else [weight_checksum(model)]
        rstats = hvd.allgather(stats) if size > 1 else [stats]
        from cori_intml_examples_amd.parallel.dist import auto_plane, data_plane
        xk = getattr(red, "xgmi_bucket", None)
        selfcheck = {
            "data_plane": (("xgmi-fused-allreduce+optim" if len(red.buckets) == 1 else
                            "hybrid: rccl buckets %s + xgmi-fused bucket %d" % (list(range(xk)), xk))
                           if xk is not None else
                           "rccl-native" if comm is not None else ("torch-" + str(st.backend))),
            # what a fit() / train_rpv run without the probe uses (INTML_XGMI unset)
            "default_plane": ((lambda p: "rccl-native" if p == "rccl" else p)(auto_plane(4 * model.store.numel))
                              if comm is not None else ("torch-" + str(st.backend))),
            "env_plane": data_plane(),
            "rccl_nranks": comm.nranks if comm is not None else None,
            "world_size": size,
            "bucket_bytes": [4 * (hi - lo) for lo, hi in red.buckets] if red is not None else None,
            "weights_identical": all(s == sums[0] for s in sums),
            "weight_checksum": sums[0],
            "step_ms_p50_per_rank": [round(r["p50"], 4) for r in rstats],
            "step_ms_max_per_rank": [round(r["max"], 4) for r in rstats],
            "plane_probe_ms_per_step": plane_probe,
        }
        ok = selfcheck["weights_identical"] and (comm is None or selfcheck["rccl_nranks"] == size)
        if not args.no_dp_delta and not args.via_fit:
            # the same step without the data-parallel machinery, same N, right after
            ref, *_ = build(args, size, False, dev)
            data2 = synthetic(max(args.samples, B * 4), shape, ncls, ref._executor, dev, g)
            e2, _ = time_steps(ref, data2, B, args.steps, args.warmup, chunk, g, dev, settle_ms=args.settle_ms)
            if size > 1:
                e2 = max(hvd.allgather(e2))
            selfcheck["nodp_ms_per_step"] = round(e2 / args.steps * 1e3, 4)
            selfcheck["exposed_comm_us_per_step"] = round((elapsed - e2) / args.steps * 1e6, 2)
            if getattr(red, "xgmi", None) is not None:
                # the same DP step with the RCCL all-reduce + optimizer launch instead of the
                # fused xGMI kernel (comparison only; the line's value is the default path)
                old = os.environ.get("INTML_XGMI")
                os.environ["INTML_XGMI"] = "0"
                try:
                    alt, *_ = build(args, size, True, dev)
                    hvd.broadcast_global_variables(0, model=alt)
                    data3 = synthetic(max(args.samples, B * 4), shape, ncls, alt._executor, dev, g)
                    e3, _ = time_steps(alt, data3, B, args.steps, args.warmup, chunk, g, dev,
                                       settle_ms=args.settle_ms)
                finally:
                    if old is None:
                        os.environ.pop("INTML_XGMI", None)
                    else:
                        os.environ["INTML_XGMI"] = old
                if size > 1:
                    e3 = max(hvd.allgather(e3))
                selfcheck["rccl_path_ms_per_step"] = round(e3 / args.steps * 1e3, 4)

    ms = elapsed / steps * 1e3
    value = size * B * steps / elapsed
    # every rank leaves the data-parallel group; rank 0 then runs the HPO on the farm
    hvd.shutdown()
    hpo_recs = None
    if inline_hpo is not None:
        try:
            hpo_recs = inline_hpo.run()
        except Exception as e:   # noqa: BLE001
            inline_hpo.stop()
            hpo_recs = {"hpo": {"error": str(e)[:300]}}
    if rank == 0:
        out = {"metric": metric,
               "value": round(value, 1), "unit": "images/s", "n_gpus": size, "steps": steps,
               "warmup": warmup_note, "ms_per_step": round(ms, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": round(value / baseline, 2) if baseline else None,
               "dtype": "bf16", "data": "synthetic (RPV-like jets / MNIST-like templates generated on the GPU by the K16 kernel, device-resident; random-init weights)",
               "config": {"model": cfg_name, "global_batch": B * size, "per_gpu_batch": B,
                          "seq_len": None, "input": list(shape),
                          "optimizer": type(getattr(model.optimizer, "_base_optimizer", model.optimizer)).__name__,
                          "parallelism": "dp%d" % size, "steps_per_graph": chunk,
                          "path": "fit" if args.via_fit else "train_steps",
                          "step_ms_p50": round(stats["p50"], 4), "step_ms_max": round(stats["max"], 4),
                          "train_loss": round(loss, 5)}}
        if not args.via_fit:
            # untimed back-to-back replays of the timed graph after the warmup (clock settle,
            # see time_steps) -- reported, not counted as warmup
            out["settle_steps"] = settle.get("settle_steps", 0)
            out["settle_ms"] = settle.get("settle_ms", 0.0)
        if args.via_fit:
            out["data"] = "synthetic (host numpy uploaded by fit(), random-init weights)"
            out["config"]["lr_warmup_epochs"] = args.lr_warmup_epochs
        if selfcheck is not None:
            out["selfcheck"] = selfcheck
        if hpo_recs is not None:
            out.update(hpo_recs)
        print(json.dumps(out), flush=True)
    if not ok:
        print("bench self-check FAILED: %s" % json.dumps(selfcheck), file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    sys.exit(main())
