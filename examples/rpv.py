"""``from rpv import load_dataset, build_model, train_model`` as in the RPV notebooks."""
import _path  # noqa: F401
from cori_intml_examples_amd.apps.rpv import (N_TEST, N_TRAIN, N_VALID, build_model,  # noqa: F401
                                              classification_report, load_dataset, load_file, train_model)
