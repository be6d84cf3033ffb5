"""Per-workgroup start/end (wall clock) of the conv backward launches of the RPV B=128 step:
the two dual (wgrad + dgrad) launches and the first conv's wgrad.  Shows the launch config,
and for the wgrad and dgrad workgroups separately: start spread, duration, last end."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cori_intml_examples_amd.apps import zoo

os.environ["INTML_GRAPHS"] = "0"
dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
MODEL = os.environ.get("MODEL", "rpv")
rs = np.random.RandomState(0)
if MODEL == "mnist":      # DistTrain_mnist: 28x28x1, conv 32-64 + pool, fc 128, softmax 10
    model = zoo.mnist_cnn(32, 64, 128, dropout=0.4, optimizer="Adadelta", lr=1.0, input_shape=(28, 28, 1), device=dev)
    xs = rs.rand(B * 4, 28, 28, 1).astype(np.float32)
    ys = np.eye(10, dtype=np.float32)[rs.randint(0, 10, B * 4)]
else:
    model = zoo.rpv_cnn((64, 64, 3), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2, optimizer="Adam",
                        lr=1e-3, device=dev)
    xs = rs.rand(B * 4, 64, 64, 3).astype(np.float32)
    ys = (rs.rand(B * 4) > 0.5).astype(np.float32)
ex = model._executor
ex.use_graphs = False
d = ex.upload(xs, ys)
ex.train_step(d, torch.arange(d.n, device=dev), 0, B)
torch.cuda.synchronize()
bp = ex._plans[(B, "train")]
s = torch.cuda.current_stream().cuda_stream


def cdiv(a, b):
    return (a + b - 1) // b


def stats(v):
    return "med %6.2f p90 %6.2f max %6.2f" % (np.median(v), np.percentile(v, 90), v.max())


for name, fn, *_ in bp.launches:
    if not (name.startswith("wgrad_dgrad") or name.startswith("wgrad_conv")):
        continue
    dfl = fn.__defaults__
    if name.startswith("wgrad_dgrad"):
        ca, ntc, wa, cfg = dfl[:4]
    else:
        ca, ntc, (wa, cfg) = None, None, dfl[:2]
    MT, NTT, S = cfg
    n_w = S * cdiv(wa.NT, NTT) * cdiv(wa.Ktiles, MT)
    n_c = 0
    if ca is not None:
        n_c = ca.B * cdiv(ca.Ho, ca.R) * cdiv(ca.NT, ntc)
    ts = torch.zeros(2 * (n_w + n_c), dtype=torch.int64, device=dev)
    wa.ts = ts.data_ptr()
    ph2 = torch.zeros(16 * (n_w + n_c), dtype=torch.int64, device=dev)
    wa.ts2 = ph2.data_ptr()
    ph = None
    if ca is not None:
        ph = torch.zeros(8 * (n_w + n_c), dtype=torch.int64, device=dev)
        ca.ts = ph.data_ptr()
    for _ in range(10):
        fn(s)
    torch.cuda.synchronize()
    wa.ts = 0
    wa.ts2 = 0
    q = ph2.view(-1, 16).cpu().numpy().astype(np.float64)[:n_w] * 0.01
    nb = wa.blocks_per_split
    segs = ["ktab", "fetch0"] + sum([["commit%d" % k, "mma%d" % k] for k in range(nb)], [])
    idx = [0, 1] + sum([[2 + 2 * k, 3 + 2 * k] for k in range(nb)], []) + [15]
    parts = []
    for k in range(len(idx) - 1):
        d = q[:, idx[k + 1]] - q[:, idx[k]]
        d = d[(q[:, idx[k + 1]] > 0) & (q[:, idx[k]] > 0)]
        if len(d):
            parts.append("%s->%s +%.2f" % (segs[k] if k < len(segs) else "?", "slab" if idx[k + 1] == 15 else "", np.median(d)))
    print("   wgrad phases (wave 0, median us):", ", ".join(parts))
    if (q[:, 8] > 0).any():
        m = lambda a_, b_: np.median((q[:, b_] - q[:, a_])[(q[:, a_] > 0) & (q[:, b_] > 0)])
        print("   wgrad start detail: ktab+barrier %.2f, per-lane setup %.2f, fetch issue %.2f" % (
            m(0, 8), m(8, 9), m(9, 1)))
    if ca is not None:
        ca.ts = 0
        p = ph.view(-1, 8).cpu().numpy().astype(np.float64)[n_w:] * 0.01
        labels = ["weights staged", "halo staged", "barrier", "1st pass MFMA", "1st pass epilogue", "wave-0 done"]
        print("   dgrad phases (wave 0, median us):", ", ".join(
            "%s +%.2f" % (lab, np.median(p[:, i + 1] - p[:, i])) for i, lab in enumerate(labels)))
    t = ts.view(-1, 2).cpu().numpy().astype(np.float64) * 0.01
    t0 = t[:, 0].min()
    st, en = t[:, 0] - t0, t[:, 1] - t0
    du = en - st
    print("%s: wgrad R=%d bps=%d MT=%d NTT=%d S=%d Ktiles=%d NT=%d -> %d WGs" % (
        name, wa.R, wa.blocks_per_split, MT, NTT, S, wa.Ktiles, wa.NT, n_w), end="")
    if ca is not None:
        print("; dgrad R=%d ntc=%d KS=%d NT=%d Ho=%d Wo=%d -> %d WGs" % (ca.R, ntc, ca.KS, ca.NT, ca.Ho, ca.Wo, n_c))
    else:
        print()
    print("   span %.2f us" % en.max())
    for lab, sl in (("wgrad", slice(0, n_w)), ("dgrad", slice(n_w, n_w + n_c))):
        if sl.stop <= sl.start:
            continue
        print("   %s start %s | dur %s | end %s" % (lab, stats(st[sl]), stats(du[sl]), stats(en[sl])))

# A/B of dgrad-body variants inside the dual launches (ca.dbg), interleaved rounds
def _t(fn, reps=40):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn(s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


variants = [int(v) for v in os.environ.get("AB_DBG", "0,16").split(",")]
for name, fn, *_ in bp.launches:
    if not name.startswith("wgrad_dgrad"):
        continue
    ca, wa = fn.__defaults__[0], fn.__defaults__[2]
    res = {v: [] for v in variants}
    for _ in range(5):
        for v in variants:
            ca.dbg = v
            wa.dbg = v
            _t(fn, 5)
            res[v].append(_t(fn))
    ca.dbg = 0
    wa.dbg = 0
    print("%s A/B dbg (dgrad + wgrad): %s" % (name, "  ".join("%d: %.2f" % (v, np.median(res[v])) for v in variants)))
