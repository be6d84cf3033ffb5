"""DistWidgetHPO_mnist workflow: the live dashboard over a random search.  In Jupyter (with
ipywidgets/bqplot) ``display(psw)`` shows the table and curves; here the same headless
model is printed as text while the trials stream their epochs (``IPyParallelLogger``)."""
import argparse
import time
from functools import partial

from common import connect, farm_args
from cori_intml_examples_amd.hpo import random_search as rs
from cori_intml_examples_amd.widgets import ModelController, ModelPlot, ParamSpanWidget


def build_and_train(h1, h2, h3, dropout, optimizer, n_epochs=16, n_train=60000):
    from cori_intml_examples_amd.apps.mlextras import IPyParallelLogger
    from cori_intml_examples_amd.apps.mnist import build_model, load_data
    x, y, _, _ = load_data(n_train=n_train)
    model = build_model(h1=h1, h2=h2, h3=h3, dropout=dropout, optimizer=optimizer)
    return model.fit(x[:n_train], y[:n_train], batch_size=128, epochs=n_epochs, validation_split=0.17,
                     callbacks=[IPyParallelLogger()], verbose=0).history


def main():
    p = farm_args(argparse.ArgumentParser(description=__doc__))
    p.add_argument("--trials", type=int, default=8)
    p.add_argument("--epochs", type=int, default=16)
    p.add_argument("--n-train", type=int, default=60000)
    a = p.parse_args()
    trials = rs.mnist_trials(a.trials)
    params = {k: [t[k] for t in trials] for k in ("h1", "h2", "h3", "dropout", "optimizer")}
    c, cl = connect(a)
    try:
        plot = partial(ModelPlot, y=["loss", "acc", "val_loss", "val_acc"], x="epoch", xlim=[0, a.epochs])
        psw = ParamSpanWidget(partial(build_and_train, n_epochs=a.epochs, n_train=a.n_train), plot, params,
                              controller=ModelController(client=c))
        psw.submit_computations(poll=False)
        while not psw.wait(timeout=5):
            print(psw.table[["status", "epoch", "h1", "h2", "h3", "val_acc"]].to_string(), "\n", flush=True)
        print(psw.render())
        i = int(psw.table.val_acc.astype(float).idxmax())
        print("best trial %d: %s" % (i, rs.describe(trials[i])))
    finally:
        c.close()
        if cl:
            cl.stop()


if __name__ == "__main__":
    main()
