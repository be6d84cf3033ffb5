"""Worker for tests/test_dp.py::test_fit_detects_divergent_rank (gloo, CPU): fit() with the
Horovod optimizer checks a cross-rank weight digest at every epoch end (train.loop.
dp_consistency_check).  Scenario "ok": the ranks stay identical and every epoch's record says
so.  Scenario "diverge": rank 1 perturbs one weight at the start of epoch 1 (what an ordering
bug in a data plane would do silently); fit() must raise DataParallelDivergence on EVERY rank
at the end of that epoch, and the History must hold the failing record."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cori_intml_examples_amd.apps import zoo  # noqa: E402
from cori_intml_examples_amd.io.datasets import synthetic_rpv  # noqa: E402
from cori_intml_examples_amd.parallel import hvd  # noqa: E402
from cori_intml_examples_amd.train import callbacks as cbks  # noqa: E402


class Perturb(cbks.Callback):
    def __init__(self, epoch):
        super().__init__()
        self.epoch = epoch

    def on_epoch_begin(self, epoch, logs=None):
        if epoch == self.epoch:
            self.model.store.master[3] += 1e-3       # one weight, one rank


def main(out_dir, scenario):
    hvd.init()
    r = hvd.rank()
    m = zoo.rpv_cnn((16, 16, 1), conv_sizes=[4, 8, 8], fc_sizes=[16], dropout=0.0, optimizer="Adam",
                    lr=0.01, use_horovod=True, device="cpu")
    hvd.broadcast_model_state(m, 0)
    x, y, _ = synthetic_rpv(64, size=16, seed=7)
    cb = [hvd.callbacks.BroadcastGlobalVariablesCallback(0)]
    if scenario == "diverge" and r == 1:
        cb.append(Perturb(1))
    rep = {"rank": r, "raised": None}
    try:
        m.fit(x, y, batch_size=16, epochs=3, verbose=0, callbacks=cb)
    except hvd.DataParallelDivergence as e:
        rep["raised"] = str(e)
    rep["records"] = m.history.dp_consistency
    rep["epochs_done"] = len(m.history.history.get("loss", []))
    with open(os.path.join(out_dir, "div%d.json" % r), "w") as f:
        json.dump(rep, f)
    hvd.shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
