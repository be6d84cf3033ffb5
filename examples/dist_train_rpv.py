"""DistTrain_rpv workflow: data-parallel RPV classifier over the farm engines, then the
notebook's analysis: pull the history from the engines (``c[0].get('history.epoch')``,
``c[:].get('history.history')``), predict on the test set on the engines, and compute
accuracy / purity / efficiency and the ROC AUC on the client (``DistTrain_rpv.ipynb``)."""
import argparse

import numpy as np

from common import connect, farm_args
from cori_intml_examples_amd.farm.magics import px


def main():
    p = farm_args(argparse.ArgumentParser(description=__doc__))
    p.add_argument("--input-dir", default="/nonexistent")
    p.add_argument("--n-train", type=int, default=64000)
    p.add_argument("--n-valid", type=int, default=32000)
    p.add_argument("--n-test", type=int, default=32000)
    p.add_argument("--epochs", type=int, default=4)
    p.add_argument("--batch-size", type=int, default=128)
    a = p.parse_args()
    c, cl = connect(a)
    try:
        px("""
from cori_intml_examples_amd.apps.rpv import load_dataset, build_model, train_model
from cori_intml_examples_amd.parallel import hvd
hvd.init()
train, valid, test = load_dataset(%r, %d, %d, %d, synthetic=True)
model = build_model(train[0].shape[1:], conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2,
                    optimizer='Adam', lr=0.001 * hvd.size(), use_horovod=True)
if hvd.rank() == 0:
    model.summary()
history = train_model(model, train[0], train[1], valid[0], valid[1], batch_size=%d, n_epochs=%d,
                      use_horovod=True, verbose=2)
test_output = model.predict(test[0], batch_size=1024)
""" % (a.input_dir, a.n_train, a.n_valid, a.n_test, a.batch_size, a.epochs), client=c)
        epochs = c[0].get("history.epoch")
        hists = c[:].get("history.history")
        print("epochs:", epochs)
        print("rank-0 val_loss:", hists[0]["val_loss"])
        out = np.asarray(c[0].get("test_output")).reshape(-1)
        labels = np.asarray(c[0].get("test[1]")).reshape(-1)
        weights = np.asarray(c[0].get("test[2]")).reshape(-1)
        from cori_intml_examples_amd.apps.rpv import classification_report
        print("unweighted:", classification_report(labels, out))
        print("weighted:  ", classification_report(labels, out, weights))
        from sklearn.metrics import roc_auc_score
        print("ROC AUC: %.4f" % roc_auc_score(labels, out))
    finally:
        c.close()
        if cl:
            cl.stop()


if __name__ == "__main__":
    main()
