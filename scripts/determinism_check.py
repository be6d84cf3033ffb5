"""Bitwise run-to-run determinism of the RPV training step on one GPU: train 4 Adam steps
from identical weights three times per configuration and compare the final weights
exactly (all reductions are fixed-order by design, so any difference is a race).

    python scripts/determinism_check.py [runs]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cori_intml_examples_amd.apps import zoo  # noqa: E402
from cori_intml_examples_amd.io.datasets import synthetic_rpv  # noqa: E402


def flat(m):
    return np.concatenate([w.ravel() for w in m.get_weights()])


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    kw = dict(conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.0, optimizer="Adam", lr=1e-3, device="cuda:0")
    x, y, _ = synthetic_rpv(512, channels=3, seed=5)
    w0 = zoo.rpv_cnn((64, 64, 3), use_horovod=False, **kw).get_weights()
    ok = True
    for label, env in (("single-GPU fused", {}), ("prologue step", {"INTML_TUNE": "pro_free=0"}),
                       ("prologue re-pack", {"INTML_TUNE": "pro_free=0,opt_packs=0"}),
                       ("no early reduce", {"INTML_TUNE": "early_reduce=0"}),
                       ("graphs off", {"INTML_GRAPHS": "0"})):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        outs = []
        for _ in range(runs):
            m = zoo.rpv_cnn((64, 64, 3), use_horovod=False, **kw)
            m.set_weights(w0)
            for i in range(4):
                m.train_on_batch(x[i * 128:(i + 1) * 128], y[i * 128:(i + 1) * 128])
            torch.cuda.synchronize()
            outs.append(flat(m))
        diffs = [float(np.abs(o - outs[0]).max()) for o in outs[1:]]
        nbad = [int((o != outs[0]).sum()) for o in outs[1:]]
        print("%-18s run-to-run max|dw| %s  differing params %s" % (label, diffs, nbad), flush=True)
        if any(nbad):
            ok = False
            d = outs[1] != outs[0]
            names, off = [], 0
            for w in m.get_weights():
                n = w.size
                if d[off:off + n].any():
                    names.append((w.shape, int(d[off:off + n].sum())))
                off += n
            print("   differing tensors (shape, count):", names, flush=True)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
