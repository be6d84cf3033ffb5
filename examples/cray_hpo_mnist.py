"""CrayHPO_mnist workflow: genetic search over the MNIST CNN with ``train.py --epochs N``
as the evaluator command (one GPU per evaluation)."""
import argparse
import os

import _path  # noqa: F401
from cori_intml_examples_amd import hpo


def main():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--generations", type=int, default=16)
    p.add_argument("--demes", type=int, default=4)
    p.add_argument("--pop-size", type=int, default=4)
    p.add_argument("--epochs", type=int, default=4)
    p.add_argument("--train-args", default="")
    p.add_argument("--log", default="mnist_hpo.log")
    a = p.parse_args()
    params = hpo.Params([["--h1", 4, [4, 8, 16]],
                         ["--h2", 8, [8, 16, 32]],
                         ["--h3", 16, [16, 32, 64]],
                         ["--dropout", 0.2, (0., 1.)],
                         ["--optimizer", "Adam", ["Adam", "Nadam"]]])
    here = os.path.dirname(os.path.abspath(__file__))
    ev = hpo.Evaluator("python %s --epochs %d %s" % (os.path.join(here, "train.py"), a.epochs, a.train_args),
                       verbose=True)
    opt = hpo.genetic.Optimizer(ev, pop_size=a.pop_size, num_demes=a.demes, generations=a.generations,
                                log_fn=a.log)
    print("best:", opt.optimize(params), "FoM", opt.best_fom)


if __name__ == "__main__":
    main()
