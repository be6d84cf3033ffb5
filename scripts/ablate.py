"""Per-kernel timing + ablation of one captured training step (cori_intml_examples_amd).

For every launch of the RPV bench step: time it alone (HIP events, 50 reps, after one real
step so buffers hold realistic data).  For conv_halo / wgrad_halo launches also time the
ablated variants (dbg bits: 1 skip staging, 2 skip MFMA, 4 skip stores) -- timing only,
results are garbage -- to see which phase dominates.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cori_intml_examples_amd.apps import zoo

os.environ["INTML_GRAPHS"] = "0"
dev = torch.device("cuda", 0)
B = int(os.environ.get("ABL_BATCH", "128"))
model = zoo.rpv_cnn((64, 64, 3), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2, optimizer="Adam",
                    lr=1e-3, device=dev)
ex = model._executor
ex.use_graphs = False
rs = np.random.RandomState(0)
x = rs.rand(B * 4, 64, 64, 3).astype(np.float32)
y = (rs.rand(B * 4) > 0.5).astype(np.float32)
d = ex.upload(x, y)
perm = torch.arange(d.n, device=dev)
ex.train_step(d, perm, 0, B)
torch.cuda.synchronize()
bp = ex._plans[(B, "train")]
s = torch.cuda.current_stream().cuda_stream


def timeit(fn, reps=50):
    for _ in range(3):
        fn(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn(s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


total = 0.0
print("%-16s %9s | ablations (us): stage-off  mfma-off  store-off  all-off" % ("launch", "us"))
for item in bp.launches:
    name, fn = item[0], item[1]
    t = timeit(fn)
    total += t
    line = "%-16s %9.2f" % (name, t)
    args = fn.__defaults__[0] if fn.__defaults__ else None
    if hasattr(args, "dbg"):
        res = []
        for dbg in (1, 2, 4, 7):
            args.dbg = dbg
            res.append(timeit(fn))
        args.dbg = 0
        line += " | " + "  ".join("%9.2f" % v for v in res)
    print(line, flush=True)
K = ex.K
for gi, (lo, hi, descs) in enumerate(bp.red_groups):
    for d in descs:
        tab = K.RedTable()
        tab.add(*d)
        t = timeit(lambda st, tab=tab: K.slab_reduce(ex.store.grad.data_ptr(), 0, 0, tab, st))
        print("  reduce grp%d type%d S=%d numel=%d: %.2f us" % (gi, d[6], d[2], d[5], t))
t = timeit(lambda st: bp._launch_optim())
total += t
print("%-16s %9.2f" % ("optim", t))
print("sum %.1f us" % total)
