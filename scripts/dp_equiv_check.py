"""DP path (INTML_DP_FORCE=1, native RCCL engine at N=1) vs single-GPU step, each with the
prologue-free / optimizer-written-packs executor and with the prologue re-pack executor, from
identical weights: prints whether each path is bit-identical across the two executors and the
DP-vs-single distance.  python scripts/dp_equiv_check.py <seed>"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["INTML_DP_FORCE"] = "1"
from cori_intml_examples_amd.apps import zoo  # noqa: E402
from cori_intml_examples_amd.io.datasets import synthetic_rpv  # noqa: E402
from cori_intml_examples_amd.parallel import hvd  # noqa: E402
from cori_intml_examples_amd.utils import set_random_seed  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
hvd.init()
kw = dict(conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.0, optimizer="Adam", lr=1e-3, device="cuda:0")
x, y, _ = synthetic_rpv(512, channels=3, seed=5)
set_random_seed(seed)
w0 = zoo.rpv_cnn((64, 64, 3), use_horovod=False, **kw).get_weights()
out = {}
for dp in (False, True):
    for tv in ("", "pro_free=0,opt_packs=0"):
        os.environ["INTML_TUNE"] = tv
        m = zoo.rpv_cnn((64, 64, 3), use_horovod=dp, **kw)
        m.set_weights(w0)
        for i in range(4):
            m.train_on_batch(x[i * 128:(i + 1) * 128], y[i * 128:(i + 1) * 128])
        torch.cuda.synchronize()
        out[(dp, tv)] = np.concatenate([w.ravel() for w in m.get_weights()])
s_new, s_old = out[(False, "")], out[(False, "pro_free=0,opt_packs=0")]
d_new, d_old = out[(True, "")], out[(True, "pro_free=0,opt_packs=0")]
q = lambda a, b: (float(np.quantile(np.abs(a - b), 0.999)), float(np.abs(a - b).max()))
print("seed %d: single new==old %s, dp new==old %s, dp-vs-single p999/max new %s old %s" % (
    seed, bool(np.array_equal(s_new, s_old)), bool(np.array_equal(d_new, d_old)), q(d_new, s_new), q(d_old, s_old)))
