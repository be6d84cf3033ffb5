"""Rank worker of tests/test_convergence.py: the benchmark model trained data-parallel on 2
ranks (64 per rank = the single-process global batch of 128; linear LR scaling as in
DistTrain_rpv.ipynb:271 is NOT applied, so the global step matches the single run), with
the Horovod-style callbacks (broadcast from rank 0, metric averaging).  Writes dp<rank>.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main(kind, d):
    from cori_intml_examples_amd.parallel import hvd
    from cori_intml_examples_amd.apps import zoo
    hvd.init()
    data = np.load(os.path.join(d, "data.npz"))
    w0 = [a for _, a in sorted(np.load(os.path.join(d, "w0.npz")).items(), key=lambda kv: int(kv[0].split("_")[1]))]
    if kind == "rpv":
        m = zoo.rpv_cnn((64, 64, 3), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2, optimizer="Adam",
                        lr=1e-3, use_horovod=True, device="cuda:0")
    else:
        m = zoo.mnist_cnn(32, 64, 128, 0.25, 0.5, optimizer="Adadelta", lr=1.0, use_horovod=True, device="cuda:0")
    m.set_weights(w0)
    np.random.seed(5 + hvd.rank())
    cbs = [hvd.callbacks.BroadcastGlobalVariablesCallback(0), hvd.callbacks.MetricAverageCallback()]
    h = m.fit(data["x"], data["y"], batch_size=64, epochs=2, validation_data=(data["xv"], data["yv"]),
              verbose=0, callbacks=cbs)
    with open(os.path.join(d, "dp%d.json" % hvd.rank()), "w") as f:
        rec = {k: [float(v) for v in vals] for k, vals in h.history.items()}
        rec["reducer"] = type(m._executor.reducer).__name__
        rec["data_plane"] = getattr(h, "data_plane", None)
        json.dump(rec, f)
    hvd.shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
