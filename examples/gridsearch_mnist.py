"""GridSearchCV_mnist workflow: k-fold grid search with the sklearn wrapper
(h1 x h2 x h3 x dropout = 36 candidates x 3 folds in the notebook)."""
import argparse

import _path  # noqa: F401
import pandas as pd
from sklearn.model_selection import GridSearchCV

from cori_intml_examples_amd.apps.mnist import load_data
from cori_intml_examples_amd.apps.zoo import mnist_cnn
from cori_intml_examples_amd.hpo import KerasClassifier


def build_model(h1=4, h2=8, h3=32, dropout=0.5):
    return mnist_cnn(h1=h1, h2=h2, h3=h3, dropout=dropout, optimizer="Adadelta")


def main():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--epochs", type=int, default=16)
    p.add_argument("--n-train", type=int, default=60000)
    p.add_argument("--small-grid", action="store_true")
    a = p.parse_args()
    x, y, xt, yt = load_data(n_train=a.n_train)
    x, y = x[:a.n_train], y[:a.n_train]
    base = build_model()
    base.summary()
    grid = dict(h1=[8, 16, 32], h2=[16, 32], h3=[16, 32], dropout=[0., 0.25, 0.5])
    if a.small_grid:
        grid = dict(h1=[8, 16], dropout=[0.25])
    gs = GridSearchCV(KerasClassifier(build_fn=build_model, batch_size=128, epochs=a.epochs, verbose=0),
                      grid, verbose=2, cv=3)
    gs.fit(x, y)
    res = pd.DataFrame(gs.cv_results_)
    print(res[["params", "mean_test_score", "std_test_score", "mean_fit_time"]].to_string())
    print("best:", gs.best_params_, "test accuracy:", gs.best_estimator_.score(xt, yt))


if __name__ == "__main__":
    main()
