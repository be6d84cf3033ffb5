"""DistWidgetHPO_rpv workflow: random search of the RPV classifier monitored live.

The reference (``DistWidgetHPO_rpv.ipynb:113-125,165-168,193-222``) drew one bqplot curve
per trial and a qgrid table while 4-48 RPV trainings streamed their epochs through
``IPyParallelLogger``; everything after the widget cell was broken there.  Here the same
dashboard runs headless (text) or in Jupyter, the trials run concurrently on the farm's
engines (one per GPU, or ``--engines`` per node), Stop / Restart work (``--stop-first``
stops trial 0 after its first epoch and restarts it), the dashboard shows per-engine GPU /
HBM use, and the analysis cells that were broken there (best / worst trial, top-5,
checkpoint reload + test metrics) run on the collected histories.
"""
import argparse
import os
import tempfile
import time
from functools import partial

from common import connect, farm_args
from cori_intml_examples_amd.hpo import random_search as rs
from cori_intml_examples_amd.widgets import ModelController, ModelPlot, ParamSpanWidget


def build_and_train(conv_sizes, fc_sizes, dropout, optimizer, lr, input_dir="/nonexistent", n_train=64000,
                    n_valid=32000, batch_size=64, n_epochs=16, checkpoint_dir=None, trial_index=None, verbose=2):
    """One RPV trial; streams every epoch to the dashboard (``IPyParallelLogger``)."""
    from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger
    from cori_intml_examples_amd.apps.rpv import build_model, load_dataset, train_model
    train, valid, _ = load_dataset(input_dir, n_train, n_valid, 0, synthetic=True)
    model = build_model(train[0].shape[1:], conv_sizes=list(conv_sizes), fc_sizes=list(fc_sizes),
                        dropout=dropout, optimizer=optimizer, lr=lr)
    ck = os.path.join(checkpoint_dir, "model_%d.h5" % trial_index) if checkpoint_dir is not None else None
    h = train_model(model, train[0], train[1], valid[0], valid[1], batch_size=batch_size, n_epochs=n_epochs,
                    checkpoint_file=ck, callbacks=[IPyParallelLogger()], verbose=verbose)
    return h.history


def main():
    p = farm_args(argparse.ArgumentParser(description=__doc__))
    p.add_argument("--trials", type=int, default=8)
    p.add_argument("--epochs", type=int, default=16)
    p.add_argument("--n-train", type=int, default=64000)
    p.add_argument("--n-valid", type=int, default=32000)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--input-dir", default="/nonexistent")
    p.add_argument("--stop-first", action="store_true", help="exercise Stop + Restart on trial 0")
    a = p.parse_args()
    trials = rs.rpv_trials(a.trials)
    params = {k: [t[k] for t in trials] for k in ("conv_sizes", "fc_sizes", "dropout", "optimizer", "lr")}
    params["trial_index"] = list(range(len(trials)))       # names each trial's checkpoint
    ckdir = tempfile.mkdtemp(prefix="rpv_widget_hpo_")
    c, cl = connect(a)
    try:
        train_func = partial(build_and_train, input_dir=a.input_dir, n_train=a.n_train, n_valid=a.n_valid,
                             batch_size=a.batch_size, n_epochs=a.epochs, checkpoint_dir=ckdir, verbose=0)
        plot_func = partial(ModelPlot, y=["loss", "acc", "val_loss", "val_acc"], x="epoch", xlim=[0, a.epochs],
                            xlabel="epochs", ylabel="training metrics")
        psw = ParamSpanWidget(train_func, plot_func, params, controller=ModelController(client=c))
        psw.submit_computations(poll=False)
        stopped = not a.stop_first
        while not psw.wait(timeout=3):
            tab = psw.snapshot()
            print(tab[["status", "epoch", "conv_sizes", "optimizer", "val_acc"]].to_string(), flush=True)
            print(psw.resources_text(), "\n", flush=True)
            if not stopped and str(tab.loc[0, "epoch"]) not in ("", "nan", "None") and float(tab.loc[0, "epoch"]) >= 0:
                psw.stop_models([0])
                print("stopped trial 0; restarting it", flush=True)
                time.sleep(0.5)
                psw.restart_models([0])
                stopped = True
        print(psw.render())
        hists = [f.get() if f is not None else None for f in psw.results]
        best_scores = [max(h["val_acc"]) if h else float("nan") for h in hists]
        order = sorted(range(len(hists)), key=lambda i: -best_scores[i] if best_scores[i] == best_scores[i] else 1)
        i_best, i_worst = order[0], order[-1]
        print("best trial %d: val_acc %.4f  %s" % (i_best, best_scores[i_best], rs.describe(trials[i_best])))
        print("worst trial %d: val_acc %.4f  %s" % (i_worst, best_scores[i_worst], rs.describe(trials[i_worst])))
        for i in order[:5]:
            print("  top trial %2d val_acc %.4f" % (i, best_scores[i]))
        from cori_intml_examples_amd.apps.rpv import classification_report, load_dataset
        from cori_intml_examples_amd.models import load_model
        ck = os.path.join(ckdir, "model_%d.h5" % i_best)
        _, _, test = load_dataset(a.input_dir, 0, 0, max(256, a.n_valid // 4), synthetic=True)
        model = load_model(ck)
        print("best model test metrics:", classification_report(test[1], model.predict(test[0], batch_size=1024),
                                                                 test[2]))
    finally:
        c.close()
        if cl:
            cl.stop()


if __name__ == "__main__":
    main()
