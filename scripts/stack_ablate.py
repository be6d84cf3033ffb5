"""Phase ablation of every launch of one RPV training step (timing only: ablated launches
compute garbage).  For each launch whose argument structs carry a ``dbg`` field, time it
with each ablation bit set on ALL its structs (conv_stack: 1 no MFMA loop, 2 no epilogue,
4 no global stores, 8 no staging; conv/dual halo: 1 no staging, 2 no MFMA, 4 no stores;
wgrad: 1 no staging, 2 no MFMA, 4 no slab stores).  HIP events, median of 5 x 40 reps.

    python scripts/stack_ablate.py [batch]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cori_intml_examples_amd.apps import zoo

os.environ["INTML_GRAPHS"] = "0"
dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
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


total = 0.0
print("%-20s %8s | %8s %8s %8s %8s %8s" % ("launch", "us", "dbg1", "dbg2", "dbg4", "dbg8", "all"))
for item in bp.launches:
    name, fn = item[0], item[1]
    t = timeit(fn)
    total += t
    line = "%-20s %8.2f" % (name, t)
    structs = [v for v in (fn.__defaults__ or ()) if hasattr(v, "dbg")]
    if structs:
        res = []
        for dbg in (1, 2, 4, 8, 15):
            for a in structs:
                a.dbg = dbg
            res.append(timeit(fn))
        for a in structs:
            a.dbg = 0
        line += " | " + " ".join("%8.2f" % v for v in res)
    print(line, flush=True)
print("sum %.1f us (launches timed alone, back to back)" % total)
