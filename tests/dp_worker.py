"""Worker for tests/test_dp.py: runs under ``torch.distributed.run`` (gloo, CPU) and writes
one JSON report per rank.  Invariants (SURVEY.md §4.3 "Distributed tests without a
cluster"): allreduce == sum, broadcast overwrites divergent init, identical params across
ranks after k steps, DP step == single-process step on the concatenated batch."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cori_intml_examples_amd.apps import zoo  # noqa: E402
from cori_intml_examples_amd.io.datasets import synthetic_rpv  # noqa: E402
from cori_intml_examples_amd.parallel import hvd  # noqa: E402
from cori_intml_examples_amd.utils import set_random_seed  # noqa: E402


def main(out_dir):
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    rep = {"rank": r, "size": n}
    # collectives
    rep["allreduce_sum"] = float(hvd.allreduce(torch.tensor([float(r + 1)]), average=False)[0])
    rep["allreduce_avg"] = float(hvd.allreduce(float(r + 1)))
    rep["allgather"] = hvd.allgather(r * 10)
    t = torch.full((4,), float(r))
    hvd.broadcast(t, 1)
    rep["broadcast"] = t.tolist()
    rep["broadcast_object"] = hvd.broadcast_object({"from": r}, 0)

    # divergent init -> BroadcastGlobalVariables makes it identical
    set_random_seed(1000 + r)
    m = zoo.rpv_cnn((16, 16, 1), conv_sizes=[4, 8, 8], fc_sizes=[16], dropout=0.0, optimizer="Adam",
                    lr=0.01, use_horovod=True, device="cpu")
    w_before = np.concatenate([w.reshape(-1) for w in m.get_weights()])
    rep["init_differs"] = float(np.abs(np.asarray(hvd.allgather(w_before[:8].tolist())[0]) - w_before[:8]).max())
    hvd.broadcast_model_state(m, 0)
    w0 = [w.copy() for w in m.get_weights()]

    # one DP step: rank r trains on its own 8-sample slice of an 8*n-sample batch
    per = 8
    x, y, _ = synthetic_rpv(per * n, size=16, seed=5)
    xs, ys = x[r * per:(r + 1) * per], y[r * per:(r + 1) * per]
    m.train_on_batch(xs, ys)
    red = m._executor.reducer
    rep["buckets"] = [list(b) for b in red.buckets]
    rep["numel"] = m.store.numel
    w1 = np.concatenate([w.reshape(-1) for w in m.get_weights()])
    rep["w1_digest"] = [float(w1.sum()), float(np.abs(w1).sum())]
    if r == 0:
        # single-process reference: same init, plain Adam, the whole 32-sample batch
        ref = zoo.rpv_cnn((16, 16, 1), conv_sizes=[4, 8, 8], fc_sizes=[16], dropout=0.0, optimizer="Adam",
                          lr=0.01, use_horovod=False, device="cpu")
        ref.set_weights(w0)
        ref.train_on_batch(x, y)
        wr = np.concatenate([w.reshape(-1) for w in ref.get_weights()])
        rep["dp_vs_single_maxdiff"] = float(np.abs(wr - w1).max())

    # a few epochs of fit with the reference's callbacks: ranks stay in lockstep
    from cori_intml_examples_amd.apps.rpv import train_model
    xt, yt, _ = synthetic_rpv(64, size=16, seed=7 + r)          # per-rank data
    xv, yv, _ = synthetic_rpv(32, size=16, seed=99)
    h = train_model(m, xt, yt, xv, yv, batch_size=16, n_epochs=2, use_horovod=True, verbose=0)
    wf = np.concatenate([w.reshape(-1) for w in m.get_weights()])
    rep["wf_digest"] = [float(wf.sum()), float(np.abs(wf).sum())]
    rep["val_loss"] = h.history["val_loss"]
    rep["loss"] = h.history["loss"]
    rep["history_keys"] = sorted(h.history.keys())
    with open(os.path.join(out_dir, "rank%d.json" % r), "w") as f:
        json.dump(rep, f)
    hvd.shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
