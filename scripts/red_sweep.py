"""Slab-reduction geometry sweep: for every reduction descriptor of the RPV B=128 step, time
slab_reduce alone at each threads-per-element choice (HIP events, median of 5 x 40)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cori_intml_examples_amd.apps import zoo

os.environ["INTML_GRAPHS"] = "0"
dev = torch.device("cuda", 0)
B = 128
model = zoo.rpv_cnn((64, 64, 3), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2, optimizer="Adam",
                    lr=1e-3, device=dev)
ex = model._executor
ex.use_graphs = False
rs = np.random.RandomState(0)
d = ex.upload(rs.rand(B * 4, 64, 64, 3).astype(np.float32), (rs.rand(B * 4) > 0.5).astype(np.float32))
ex.train_step(d, torch.arange(d.n, device=dev), 0, B)
torch.cuda.synchronize()
bp = ex._plans[(B, "train")]
s = torch.cuda.current_stream().cuda_stream
K = ex.K


def timeit(fn, reps=40):
    for _ in range(3):
        fn(s)
    res = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn(s)
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / reps * 1e3)
    return float(np.median(res))


for name, fn, *_ in bp.launches:
    if name.startswith("reduce"):
        print("%s (as captured): %.2f us" % (name, timeit(fn)))
for gi, (lo, hi, descs) in enumerate(bp.red_groups):
    for dsc in descs:
        row = []
        for tpe in (1, 4, 8, 16, 32, 64, 128, 256):
            if tpe > 1 and tpe > 4 * dsc[2]:
                continue
            tab = K.RedTable()
            tab.add(*dsc, tpe=tpe)
            t = timeit(lambda st, tab=tab: K.slab_reduce(ex.store.grad.data_ptr(), 0, 0, tab, st))
            row.append("%d:%.2f" % (tpe, t))
        print("grp%d type%d S=%d numel=%d  tpe:us  %s" % (gi, dsc[6], dsc[2], dsc[5], "  ".join(row)), flush=True)

# fused reduce+optimizer launch over subsets of the descriptors
descs = [d for (_, _, ds) in bp.red_groups for d in ds]
oa = ex._optim_args(False, defer_pack=True)


def table(sel):
    tab = K.RedTable()
    for d in sorted(sel, key=lambda d: -d[2]):
        tab.add(*d)
    return tab


for label, sel in (("all", descs), ("no dense W", [d for d in descs if d[6] != 2]),
                   ("dense W only", [d for d in descs if d[6] == 2]),
                   ("conv W only", [d for d in descs if d[6] == 0])):
    tab = table(sel)
    t = timeit(lambda st, tab=tab: K.reduce_optim(ex.store.grad.data_ptr(), tab, oa, st))
    print("reduce_optim [%s] %d WGs: %.2f us" % (label, tab.nblocks if hasattr(tab, "nblocks") else -1, t), flush=True)
