"""``from mnist import load_data, build_model`` as in the MNIST HPO notebooks."""
import _path  # noqa: F401
from cori_intml_examples_amd.apps.mnist import build_model, img_cols, img_rows, load_data, n_classes  # noqa: F401
