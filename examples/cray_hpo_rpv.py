"""CrayHPO_rpv workflow: genetic search where every evaluation is itself a data-parallel
``train_rpv`` run on a slice of the node's GPUs (HPO x DP).  ``--gpus-per-eval 4`` on 8
MI355X runs two 4-rank evaluations at a time (the notebook ran 8 x 4-node ones on 32
Cori nodes).  Writes the summary log and one ``Deme<d>_<log>`` per deme."""
import argparse
import os

import _path  # noqa: F401
from cori_intml_examples_amd import hpo


def main():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--generations", type=int, default=4)
    p.add_argument("--demes", type=int, default=4)
    p.add_argument("--pop-size", type=int, default=8)
    p.add_argument("--mutation-rate", type=float, default=0.05)
    p.add_argument("--crossover-rate", type=float, default=0.33)
    p.add_argument("--gpus-per-eval", type=int, default=1)
    p.add_argument("--n-epochs", type=int, default=4)
    p.add_argument("--train-args", default="", help="extra train_rpv flags, e.g. '--n-train 8000'")
    p.add_argument("--log", default="rpv_hpo.log")
    a = p.parse_args()
    params = hpo.Params([
        ["--h1", 16, (4, 64)],
        ["--h2", 32, (4, 64)],
        ["--h3", 64, (8, 128)],
        ["--h4", 128, (32, 256)],
        ["--dropout", 0.2, (0., 1.)],
        ["--optimizer", "Adam", ["Adam", "Nadam", "Adadelta"]],
        ["--lr", 1e-3, [1e-1, 1e-2, 1e-3, 1e-4, 1e-5]],
    ])
    here = os.path.dirname(os.path.abspath(__file__))
    cmd = "python %s --n-epochs %d --fom best %s" % (os.path.join(here, "train_rpv.py"), a.n_epochs, a.train_args)
    evaluator = hpo.Evaluator(cmd, gpus_per_eval=a.gpus_per_eval, verbose=True)
    print(evaluator)
    opt = hpo.GeneticOptimizer(evaluator, generations=a.generations, num_demes=a.demes, pop_size=a.pop_size,
                               mutation_rate=a.mutation_rate, crossover_rate=a.crossover_rate, verbose=True,
                               log_fn=a.log)
    best = opt.optimize(params)
    print("best FoM %.6g with %s" % (opt.best_fom, best))


if __name__ == "__main__":
    main()
