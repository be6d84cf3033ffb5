"""GPU worker for tests/test_gpu_integration.py: 2 ranks on ONE MI355X.  RCCL needs one GPU
per rank, so dist.init selects the RCCL-free xGMI data plane on its own (more local ranks than
GPUs): NativeGradReducer with the fused all-reduce + optimizer kernel captured into the step
graph -- the reducer an 8-GPU job runs when the probe picks xGMI.  Checks lockstep and
equivalence with a single-process global batch, through train_on_batch AND fit()."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cori_intml_examples_amd.apps import zoo  # noqa: E402
from cori_intml_examples_amd.io.datasets import synthetic_rpv  # noqa: E402
from cori_intml_examples_amd.parallel import hvd  # noqa: E402
from cori_intml_examples_amd.utils import set_random_seed  # noqa: E402


def flat(m):
    return np.concatenate([w.reshape(-1) for w in m.get_weights()])


def main(out_dir):
    hvd.init()
    r = hvd.rank()
    set_random_seed(10 + r)
    kw = dict(conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.0, optimizer="SGD", lr=0.05, device="cuda:0")
    m = zoo.rpv_cnn((64, 64, 3), use_horovod=True, **kw)
    hvd.broadcast_model_state(m, 0)
    w0 = m.get_weights()
    x, y, _ = synthetic_rpv(256, channels=3, seed=3)
    rep = {"rank": r}
    m.train_on_batch(x[r * 128:(r + 1) * 128], y[r * 128:(r + 1) * 128])
    w1 = flat(m)
    rep["w1"] = [float(w1.sum()), float(np.abs(w1).sum())]
    if r == 0:
        ref = zoo.rpv_cnn((64, 64, 3), use_horovod=False, **kw)
        ref.set_weights(w0)
        ref.train_on_batch(x, y)
        d = flat(ref) - w1
        step = flat(ref) - np.concatenate([w.reshape(-1) for w in w0])
        rep["rel_diff"] = float(np.linalg.norm(d) / max(np.linalg.norm(step), 1e-30))
    from cori_intml_examples_amd.apps.rpv import train_model
    xt, yt, _ = synthetic_rpv(512, channels=3, seed=7 + r)
    xv, yv, _ = synthetic_rpv(256, channels=3, seed=99)
    h = train_model(m, xt, yt, xv, yv, batch_size=128, n_epochs=2, use_horovod=True, verbose=0)
    wf = flat(m)
    rep["wf"] = [float(wf.sum()), float(np.abs(wf).sum())]
    rep["val_loss"] = h.history["val_loss"]
    rep["reducer"] = type(m._executor.reducer).__name__
    rep["data_plane"] = getattr(h, "data_plane", None)
    with open(os.path.join(out_dir, "rank%d.json" % r), "w") as f:
        json.dump(rep, f)
    hvd.shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
