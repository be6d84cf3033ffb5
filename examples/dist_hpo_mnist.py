"""DistHPO_mnist workflow: random search of the MNIST CNN over the farm (one trial per
engine / MI355X at a time), per-trial checkpoints, best-trial reload and test evaluation
(``DistHPO_mnist.ipynb``).  ``--trials 32 --epochs 16`` reproduces the notebook's search;
trial lists are identical to the notebook's for the same seed."""
import argparse
import os
import tempfile

from common import connect, farm_args
from cori_intml_examples_amd.hpo import random_search as rs


def build_and_train(h1, h2, h3, dropout, optimizer, trial_index=0, checkpoint_dir=None, batch_size=128,
                    n_epochs=16, valid_frac=0.17, n_train=60000):
    # imports inside the function: it runs on the engines (DistHPO_mnist.ipynb:169-191)
    from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger, configure_session
    from cori_intml_examples_amd.apps.mnist import build_model, load_data
    from cori_intml_examples_amd.train.callbacks import ModelCheckpoint
    configure_session()
    x_train, y_train, _, _ = load_data(n_train=n_train)
    x_train, y_train = x_train[:n_train], y_train[:n_train]
    model = build_model(h1=h1, h2=h2, h3=h3, dropout=dropout, optimizer=optimizer)
    cbs = [IPyParallelLogger()]
    if checkpoint_dir:
        cbs.append(ModelCheckpoint(os.path.join(checkpoint_dir, "model_%i.h5" % trial_index)))
    history = model.fit(x_train, y_train, batch_size=batch_size, epochs=n_epochs, validation_split=valid_frac,
                        callbacks=cbs, verbose=2)
    return history.history


def main():
    p = farm_args(argparse.ArgumentParser(description=__doc__))
    p.add_argument("--trials", type=int, default=32)
    p.add_argument("--epochs", type=int, default=16)
    p.add_argument("--n-train", type=int, default=60000)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--checkpoint-dir", default=None)
    a = p.parse_args()
    ckdir = a.checkpoint_dir or tempfile.mkdtemp(prefix="mnist_hpo_")
    trials = rs.mnist_trials(a.trials, a.seed)
    for i, t in enumerate(trials):
        print("Trial %i: %s" % (i, rs.describe(t)))
    c, cl = connect(a)
    try:
        lv = c.load_balanced_view()
        ars = rs.submit_trials(lv, build_and_train, trials, with_index=True, checkpoint_dir=ckdir,
                               n_epochs=a.epochs, n_train=a.n_train)
        rs.wait_progress(ars, interval=2.0)
        hists = rs.collect(ars)
        print("trial runtimes (s):", rs.runtime_seconds(ars).round(1).tolist())
        i, best = rs.best_trial(hists, "val_acc", "max")
        print("Best trial %d (%s): val_acc %.4f" % (i, rs.describe(trials[i]), best))
        from cori_intml_examples_amd.apps.mnist import load_data
        from cori_intml_examples_amd.models import load_model
        _, _, x_test, y_test = load_data(n_train=a.n_train)
        model = load_model(os.path.join(ckdir, "model_%i.h5" % i))
        score = model.evaluate(x_test, y_test, verbose=0)
        print("Best model test loss %.4f, accuracy %.4f" % (score[0], score[1]))
    finally:
        c.close()
        if cl:
            cl.stop()


if __name__ == "__main__":
    main()
