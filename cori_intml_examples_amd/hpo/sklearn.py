"""scikit-learn estimator wrappers (``keras.wrappers.scikit_learn``), used by the k-fold
grid search of ``GridSearchCV_mnist.ipynb:275-284``:

    sk_model = KerasClassifier(build_fn=build_model, batch_size=128, epochs=16, verbose=0)
    GridSearchCV(sk_model, dict(h1=[8,16,32], h2=[16,32], h3=[16,32], dropout=[0,.25,.5])).fit(x, y)

``build_fn`` receives the grid's hyper-parameters (those it declares); ``fit`` /
``predict`` / ``score`` receive the rest.  Semantics follow Keras 2.2's wrapper:
integer labels are one-hot encoded for a categorical cross-entropy model, ``predict``
returns class labels, ``score`` is the model's accuracy (``evaluate``'s metric).
"""
from __future__ import annotations

import copy
import inspect
from typing import Any, Dict

import numpy as np

_FIT_ARGS = ("batch_size", "epochs", "verbose", "callbacks", "validation_split", "validation_data",
             "shuffle", "initial_epoch")
_PRED_ARGS = ("batch_size", "verbose")
_EVAL_ARGS = ("batch_size", "verbose")


class BaseWrapper:
    def __init__(self, build_fn=None, **sk_params):
        self.build_fn = build_fn
        self.sk_params = sk_params
        self.check_params(sk_params)

    # -- sklearn estimator protocol ---------------------------------------------------
    def _legal(self):
        fn = self.build_fn if self.build_fn is not None else self.__call__
        names = set(inspect.signature(fn).parameters)
        return names | set(_FIT_ARGS) | set(_PRED_ARGS) | set(_EVAL_ARGS)

    def check_params(self, params):
        legal = self._legal()
        for k in params:
            if k not in legal:
                raise ValueError("{} is not a legal parameter".format(k))

    def get_params(self, deep=False, **_):
        res = copy.deepcopy(self.sk_params) if deep else dict(self.sk_params)
        res["build_fn"] = self.build_fn
        return res

    def set_params(self, **params):
        self.check_params(params)
        self.sk_params.update(params)
        return self

    def filter_sk_params(self, fn, override=None) -> Dict[str, Any]:
        override = override or {}
        names = inspect.signature(fn).parameters
        out = {k: v for k, v in self.sk_params.items() if k in names}
        out.update({k: v for k, v in override.items() if k in names})
        return out

    def __sklearn_tags__(self):
        from sklearn.base import BaseEstimator
        tags = BaseEstimator.__sklearn_tags__(self)
        kind = getattr(self, "_estimator_type", None)
        if kind == "classifier":
            from sklearn.utils import ClassifierTags
            tags.estimator_type, tags.classifier_tags = "classifier", ClassifierTags()
        elif kind == "regressor":
            from sklearn.utils import RegressorTags
            tags.estimator_type, tags.regressor_tags = "regressor", RegressorTags()
        return tags

    def _pick(self, names, kwargs):
        out = {k: v for k, v in self.sk_params.items() if k in names}
        out.update({k: v for k, v in kwargs.items() if k in names})
        return out

    # -- training -------------------------------------------------------------------------
    def fit(self, x, y, **kwargs):
        self.model = self.build_fn(**self.filter_sk_params(self.build_fn))
        loss = getattr(self.model, "loss", None)
        lname = loss if isinstance(loss, str) else getattr(loss, "__name__", "")
        y = np.asarray(y)
        if lname == "categorical_crossentropy" and y.ndim == 1:
            from ..utils import to_categorical
            y = to_categorical(y, self.model.output_shape[-1])
        fit_args = self._pick(_FIT_ARGS, kwargs)
        self.history_ = self.model.fit(x, y, **fit_args)
        return self.history_


class KerasClassifier(BaseWrapper):
    _estimator_type = "classifier"
    def fit(self, x, y, **kwargs):
        y = np.asarray(y)
        if y.ndim == 2 and y.shape[1] > 1:
            self.classes_ = np.arange(y.shape[1])
        elif y.ndim == 2 and y.shape[1] == 1 or y.ndim == 1:
            self.classes_ = np.unique(y)
            y = np.searchsorted(self.classes_, y.reshape(-1))
        else:
            raise ValueError("Invalid shape for y: " + str(y.shape))
        self.n_classes_ = len(self.classes_)
        return super().fit(x, y, **kwargs)

    def predict(self, x, **kwargs):
        classes = self.model.predict_classes(x, **self._pick(_PRED_ARGS, kwargs))
        return self.classes_[np.asarray(classes).reshape(-1)]

    def predict_proba(self, x, **kwargs):
        probs = self.model.predict(x, **self._pick(_PRED_ARGS, kwargs))
        if probs.shape[1] == 1:
            probs = np.hstack([1 - probs, probs])
        return probs

    def score(self, x, y, **kwargs):
        y = np.asarray(y)
        if y.ndim == 2 and y.shape[1] > 1:
            y = y.argmax(axis=1)
        y = np.searchsorted(self.classes_, y.reshape(-1))
        lname = self.model.loss if isinstance(self.model.loss, str) else getattr(self.model.loss, "__name__", "")
        if lname == "categorical_crossentropy":
            from ..utils import to_categorical
            y = to_categorical(y, self.n_classes_)
        out = self.model.evaluate(x, y, **self._pick(_EVAL_ARGS, dict(kwargs, verbose=kwargs.get("verbose", 0))))
        if isinstance(out, list):
            return out[1] if len(out) > 1 else -out[0]
        return -out


class KerasRegressor(BaseWrapper):
    _estimator_type = "regressor"
    def predict(self, x, **kwargs):
        return np.squeeze(self.model.predict(x, **self._pick(_PRED_ARGS, kwargs)))

    def score(self, x, y, **kwargs):
        out = self.model.evaluate(x, y, **self._pick(_EVAL_ARGS, dict(kwargs, verbose=kwargs.get("verbose", 0))))
        return -(out[0] if isinstance(out, list) else out)
