"""Train_rpv workflow: single-GPU RPV training including the legacy strided 4-conv model
(34.5M parameters, ``Train_rpv.ipynb:205-219``) with a progress bar (verbose=1), then the
test metrics."""
import argparse

import _path  # noqa: F401
from cori_intml_examples_amd.apps.rpv import classification_report, load_dataset, train_model
from cori_intml_examples_amd.apps.zoo import rpv_cnn, rpv_legacy_cnn


def main():
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("--input-dir", default="/nonexistent")
    p.add_argument("--n-train", type=int, default=64000)
    p.add_argument("--n-valid", type=int, default=32000)
    p.add_argument("--n-test", type=int, default=32000)
    p.add_argument("--epochs", type=int, default=8)
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--legacy", action="store_true", help="the 34.5M-parameter strided model")
    a = p.parse_args()
    train, valid, test = load_dataset(a.input_dir, a.n_train, a.n_valid, a.n_test, synthetic=True)
    shape = train[0].shape[1:]
    model = rpv_legacy_cnn(shape) if a.legacy else rpv_cnn(shape, [16, 32, 64], [128], dropout=0.2)
    model.summary()
    train_model(model, train[0], train[1], valid[0], valid[1], a.batch_size, a.epochs, verbose=1)
    out = model.predict(test[0], batch_size=1024)
    print("test:", model.evaluate(test[0], test[1], verbose=0))
    print("unweighted:", classification_report(test[1], out))
    print("weighted:  ", classification_report(test[1], out, test[2]))


if __name__ == "__main__":
    main()
