"""Hyper-parameter optimisation: random search over the farm, Cray-HPO-style genetic search
over GPU-slot evaluations (HPO x DP), and scikit-learn wrappers for grid search.

``from cori_intml_examples_amd import hpo`` offers the ``crayai.hpo`` call shapes used by
``CrayHPO_rpv.ipynb`` (``hpo.Params``, ``hpo.Evaluator``, ``hpo.GeneticOptimizer``,
``hpo.genetic.Optimizer``)."""
from . import genetic, random_search
from .evaluator import Evaluator, parse_fom
from .genetic import GeneticOptimizer
from .params import Params
from .sklearn import KerasClassifier, KerasRegressor

__all__ = ["Params", "Evaluator", "GeneticOptimizer", "genetic", "random_search", "parse_fom",
           "KerasClassifier", "KerasRegressor"]
