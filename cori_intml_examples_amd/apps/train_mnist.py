"""MNIST training CLI with the FoM protocol -- the evaluator command of the Cray MNIST
genetic search (``python train.py --epochs N``, ``CrayHPO_mnist.ipynb:75-76``; that
script is referenced but absent from the reference repo).  Flags follow the search space
of ``CrayHPO_mnist.ipynb:41-45`` (``--h1 --h2 --h3 --dropout --optimizer``); prints
``FoM: <min val_loss>`` (lower is better).  Data-parallel under torchrun like train_rpv.
"""
from __future__ import annotations

import argparse
import sys


def build_parser():
    p = argparse.ArgumentParser(description="MNIST CNN training (FoM protocol)")
    p.add_argument("--epochs", type=int, default=4)
    p.add_argument("--h1", type=int, default=4)
    p.add_argument("--h2", type=int, default=8)
    p.add_argument("--h3", type=int, default=16)
    p.add_argument("--dropout", type=float, default=0.2)
    p.add_argument("--optimizer", default="Adam")
    p.add_argument("--lr", type=float, default=None)
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--valid-frac", type=float, default=0.17)
    p.add_argument("--n-train", type=int, default=60000)
    p.add_argument("--fom", choices=["best", "last"], default="best")
    p.add_argument("--verbose", type=int, default=2)
    return p


def main(argv=None):
    a = build_parser().parse_args(argv)
    from ..parallel import hvd
    from .mnist import load_data
    from .zoo import mnist_cnn
    hvd.init()
    x, y, _, _ = load_data(n_train=a.n_train)
    x, y = x[:a.n_train], y[:a.n_train]
    model = mnist_cnn(h1=a.h1, h2=a.h2, h3=a.h3, dropout=a.dropout, optimizer=a.optimizer, lr=a.lr,
                      use_horovod=hvd.size() > 1)
    cbs = []
    if hvd.size() > 1:
        cbs = [hvd.callbacks.BroadcastGlobalVariablesCallback(0), hvd.callbacks.MetricAverageCallback()]
    h = model.fit(x, y, batch_size=a.batch_size, epochs=a.epochs, validation_split=a.valid_frac,
                  verbose=a.verbose if hvd.rank() == 0 else 0, callbacks=cbs)
    from ..hpo.evaluator import figure_of_merit
    print("FoM:", figure_of_merit(h.history["val_loss"], a.fom))
    sys.stdout.flush()
    hvd.shutdown()
    return h


if __name__ == "__main__":
    main()
