"""Island-model genetic optimizer (``hpo.GeneticOptimizer`` / ``hpo.genetic.Optimizer``,
``CrayHPO_rpv.ipynb:161-189``, ``CrayHPO_mnist.ipynb:86-90``).

* ``num_demes`` islands of ``pop_size`` individuals each.  Generation 0 of every deme is
  the default point plus mutated copies of it (the reference's logs show generation-0
  individuals scattered around the defaults, ``CrayHPO_rpv.ipynb:1282``).
* Each generation evaluates every individual of every deme in ONE evaluator batch, so
  all GPU slots stay busy (``Evaluator.evaluate`` runs them concurrently).
* Lower FoM is better.  Per deme, fitness maps FoM linearly onto [0, 1] (1 = best,
  failed evaluations 0), matching the fitness column of the reference's deme logs.
* Next generation per deme: the best individual survives (elitism); the rest are
  tournament-selected parents, uniformly crossed over with probability
  ``crossover_rate`` and mutated gene-wise with probability ``mutation_rate``.
  Every ``migration_interval`` generations each deme's best replaces the worst of the
  next deme (ring migration).

Logs: ``log_fn`` gets one whitespace-delimited row per
generation -- ``generation epoch best_fom avg_fom checkpoint_in checkpoint_out --<hp>...``
with the best-so-far point -- and ``Deme<d>_<log_fn>`` one row per evaluation --
``generation tag fitness FoM --<hp>...``.  Rows are flushed as each generation ends
(the reference dumped the deme files only when the optimizer was deleted).
"""
from __future__ import annotations

import math
import os
from typing import Any, Dict, List, Optional

import numpy as np

from .evaluator import Evaluator
from .params import Params


def _fitness(foms: List[float]) -> List[float]:
    fin = [f for f in foms if math.isfinite(f)]
    if not fin:
        return [0.0] * len(foms)
    lo, hi = min(fin), max(fin)
    out = []
    for f in foms:
        if not math.isfinite(f):
            out.append(0.0)
        elif hi == lo:
            out.append(1.0)
        else:
            out.append((hi - f) / (hi - lo))
    return out


class GeneticOptimizer:
    def __init__(self, evaluator: Evaluator, generations: int = 10, num_demes: int = 1, pop_size: int = 8,
                 mutation_rate: float = 0.05, crossover_rate: float = 0.33, migration_interval: int = 1,
                 tournament_size: int = 2, verbose: bool = False, log_fn: str = "genetic.log",
                 seed: Optional[int] = None, init_mutation_rate: float = 0.5, mutation_scale: float = 0.1):
        self.evaluator = evaluator
        self.generations, self.num_demes, self.pop_size = int(generations), int(num_demes), int(pop_size)
        self.mutation_rate, self.crossover_rate = float(mutation_rate), float(crossover_rate)
        self.migration_interval = max(1, int(migration_interval))
        self.tournament_size = max(1, int(tournament_size))
        self.verbose, self.log_fn = verbose, log_fn
        self.init_mutation_rate, self.mutation_scale = init_mutation_rate, mutation_scale
        self.rng = np.random.RandomState(seed)
        self.best_fom = float("inf")
        self.best_params: Optional[Dict[str, Any]] = None
        self.summary: List[Dict[str, Any]] = []
        self.results: List[Dict[str, Any]] = []

    # -- bookkeeping -----------------------------------------------------------------
    def _deme_log(self, d: int) -> str:
        head, tail = os.path.split(self.log_fn)
        return os.path.join(head, "Deme%d_%s" % (d + 1, tail))

    def _write_headers(self, params: Params):
        hps = " ".join(params.flags)
        with open(self.log_fn, "w") as f:
            f.write("generation epoch best_fom avg_fom checkpoint_in checkpoint_out %s\n" % hps)
        for d in range(self.num_demes):
            with open(self._deme_log(d), "w") as f:
                f.write("generation tag fitness FoM %s\n" % hps)

    @staticmethod
    def _fmt(v) -> str:
        if isinstance(v, float):
            return "%.6g" % v
        return str(v)

    # -- evolution ---------------------------------------------------------------------
    def _initial(self, params: Params) -> List[List[Dict[str, Any]]]:
        demes = []
        base = params.defaults()
        for _ in range(self.num_demes):
            pop = [dict(base)]
            while len(pop) < self.pop_size:
                pop.append(params.mutate(base, self.rng, self.init_mutation_rate, self.mutation_scale))
            demes.append(pop)
        return demes

    def _select(self, pop, fit):
        idx = self.rng.randint(len(pop), size=self.tournament_size)
        return pop[max(idx, key=lambda i: fit[i])]

    def _next(self, params: Params, pop, fit):
        order = np.argsort(fit)[::-1]
        new = [dict(pop[order[0]])]                      # elitism
        while len(new) < self.pop_size:
            a = self._select(pop, fit)
            child = params.crossover(a, self._select(pop, fit), self.rng) if self.rng.rand() < self.crossover_rate \
                else dict(a)
            new.append(params.mutate(child, self.rng, self.mutation_rate, self.mutation_scale))
        return new

    def optimize(self, params: Params) -> Dict[str, Any]:
        self._write_headers(params)
        demes = self._initial(params)
        counters = [0] * self.num_demes
        for gen in range(self.generations):
            points, tags, where = [], [], []
            for d, pop in enumerate(demes):
                for i, ind in enumerate(pop):
                    tags.append("deme%d_ind%d" % (d + 1, counters[d]))
                    counters[d] += 1
                    points.append(params.to_args(ind))
                    where.append((d, i))
            foms = self.evaluator.evaluate(points, tags)
            per_deme: List[List[float]] = [[0.0] * len(p) for p in demes]
            for (d, i), f in zip(where, foms):
                per_deme[d][i] = f
            fits = [_fitness(fl) for fl in per_deme]
            k = 0
            for d, pop in enumerate(demes):
                with open(self._deme_log(d), "a") as fh:
                    for i, ind in enumerate(pop):
                        row = {"generation": gen, "tag": tags[k], "fitness": fits[d][i], "FoM": per_deme[d][i]}
                        row.update(ind)
                        self.results.append(row)
                        fh.write(" ".join([str(gen), tags[k], "%.6f" % fits[d][i], self._fmt(per_deme[d][i])] +
                                          [self._fmt(ind[fl]) for fl in params.flags]) + "\n")
                        k += 1
                        if per_deme[d][i] < self.best_fom:
                            self.best_fom, self.best_params = per_deme[d][i], dict(ind)
            fin = [f for f in foms if math.isfinite(f)]
            avg = float(np.mean(fin)) if fin else float("inf")
            srow = {"generation": gen, "epoch": gen + 1, "best_fom": self.best_fom, "avg_fom": avg}
            srow.update(self.best_params or {})
            self.summary.append(srow)
            with open(self.log_fn, "a") as fh:
                fh.write(" ".join([str(gen), str(gen + 1), self._fmt(self.best_fom), self._fmt(avg), "nan", "nan"] +
                                  [self._fmt((self.best_params or params.defaults())[fl]) for fl in params.flags])
                         + "\n")
            if self.verbose:
                print("generation %d: best FoM %.6g, avg FoM %.6g, best %s" % (gen, self.best_fom, avg,
                                                                               self.best_params), flush=True)
            if gen + 1 < self.generations:
                bests = [dict(pop[int(np.argmax(fits[d]))]) for d, pop in enumerate(demes)]
                demes = [self._next(params, pop, fits[d]) for d, pop in enumerate(demes)]
                if self.num_demes > 1 and (gen + 1) % self.migration_interval == 0:
                    for d in range(self.num_demes):
                        tgt = demes[(d + 1) % self.num_demes]
                        tgt[-1] = bests[d]               # replace a non-elite slot
        return dict(self.best_params or params.defaults())


Optimizer = GeneticOptimizer
