"""``python train.py --epochs N [--h1 ..]`` -- MNIST evaluator of the Cray MNIST search."""
import _path  # noqa: F401
from cori_intml_examples_amd.apps.train_mnist import main

if __name__ == "__main__":
    main()
