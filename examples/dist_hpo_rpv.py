"""DistHPO_rpv workflow: random search of the RPV classifier (conv / fc sizes, lr,
dropout, optimizer) over the farm, checkpoints per trial, the runtime histogram data
(``completed - started``), top-5 trials and a test evaluation of the best model."""
import argparse
import os
import tempfile

from common import connect, farm_args
from cori_intml_examples_amd.hpo import random_search as rs


def build_and_train(conv_sizes, fc_sizes, lr, dropout, optimizer, trial_index=0, checkpoint_dir=None,
                    input_dir="/nonexistent", n_train=64000, n_valid=32000, batch_size=64, n_epochs=16):
    from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger
    from cori_intml_examples_amd.apps.rpv import build_model, load_dataset, train_model
    train, valid, _ = load_dataset(input_dir, n_train, n_valid, 0, synthetic=True)
    model = build_model(train[0].shape[1:], conv_sizes=conv_sizes, fc_sizes=fc_sizes, dropout=dropout,
                        optimizer=optimizer, lr=lr)
    ck = os.path.join(checkpoint_dir, "model_%i.h5" % trial_index) if checkpoint_dir else None
    h = train_model(model, train[0], train[1], valid[0], valid[1], batch_size=batch_size, n_epochs=n_epochs,
                    checkpoint_file=ck, callbacks=[IPyParallelLogger()], verbose=2)
    return h.history


def main():
    p = farm_args(argparse.ArgumentParser(description=__doc__))
    p.add_argument("--trials", type=int, default=32)
    p.add_argument("--epochs", type=int, default=16)
    p.add_argument("--n-train", type=int, default=64000)
    p.add_argument("--n-valid", type=int, default=32000)
    p.add_argument("--n-test", type=int, default=32000)
    p.add_argument("--input-dir", default="/nonexistent")
    a = p.parse_args()
    ckdir = tempfile.mkdtemp(prefix="rpv_hpo_")
    trials = rs.rpv_trials(a.trials)
    c, cl = connect(a)
    try:
        ars = rs.submit_trials(c.load_balanced_view(), build_and_train, trials, with_index=True,
                               checkpoint_dir=ckdir, input_dir=a.input_dir, n_train=a.n_train,
                               n_valid=a.n_valid, n_epochs=a.epochs)
        rs.wait_progress(ars, interval=2.0)
        hists = rs.collect(ars)
        rt = rs.runtime_seconds(ars)
        print("runtime per trial: mean %.1fs min %.1fs max %.1fs" % (rt.mean(), rt.min(), rt.max()))
        scored = sorted(((min(h["val_loss"]), i) for i, h in enumerate(hists) if h), key=lambda t: t[0])
        for v, i in scored[:5]:
            print("  trial %2d val_loss %.4f  %s" % (i, v, rs.describe(trials[i])))
        best = scored[0][1]
        from cori_intml_examples_amd.apps.rpv import classification_report, load_dataset
        from cori_intml_examples_amd.models import load_model
        _, _, test = load_dataset(a.input_dir, 0, 0, a.n_test, synthetic=True)
        model = load_model(os.path.join(ckdir, "model_%i.h5" % best))
        print("best model test:", model.evaluate(test[0], test[1], verbose=0),
              classification_report(test[1], model.predict(test[0], batch_size=1024), test[2]))
    finally:
        c.close()
        if cl:
            cl.stop()


if __name__ == "__main__":
    main()
