"""HPO_mnist workflow: serial, in-process random search (no farm), 16 trials by default."""
import argparse

import _path  # noqa: F401
from cori_intml_examples_amd.apps.mnist import build_model, load_data
from cori_intml_examples_amd.hpo import random_search as rs


def main():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--trials", type=int, default=16)
    p.add_argument("--epochs", type=int, default=16)
    p.add_argument("--n-train", type=int, default=60000)
    a = p.parse_args()
    x, y, xt, yt = load_data(n_train=a.n_train)
    x, y = x[:a.n_train], y[:a.n_train]
    trials = rs.mnist_trials(a.trials)
    hists, models = [], []
    for i, t in enumerate(trials):
        print("Trial %d: %s" % (i, rs.describe(t)), flush=True)
        m = build_model(**t)
        hists.append(m.fit(x, y, batch_size=128, epochs=a.epochs, validation_split=0.17, verbose=2).history)
        models.append(m)
    i, v = rs.best_trial(hists)
    print("Best trial %d (%s) val_acc %.4f; test %s" % (i, rs.describe(trials[i]), v,
                                                        models[i].evaluate(xt, yt, verbose=0)))


if __name__ == "__main__":
    main()
