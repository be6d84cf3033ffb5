"""In-kernel phase timeline of the layer-fused conv-stack forward (wall_clock64 stamps, 10 ns,
written by lane 0 of every wave when ConvStackArgs.ts is set).  Prints, relative to the
earliest wave start: the spread of workgroup start times, and per phase the median / max
over waves of the time that phase ended, for the RPV bench step (B=128).

    python scripts/stack_timeline.py [batch]
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
fn = [f for (n, f, *_) in bp.launches if n == "conv_stack_fwd"][0]
a = fn.__defaults__[0]
nblk = a.B * a.splits
print("conv_stack: B=%d splits=%d blocks=%d lds_bytes=%d layers=%d" % (a.B, a.splits, nblk, a.lds_bytes, a.n))
nw = ex.K.STACK_THREADS // 64                 # waves per workgroup (stamp rows per block)
ts = torch.zeros(nblk * nw * 32, dtype=torch.int64, device=dev)
a.ts = ts.data_ptr()
a.dbg = int(os.environ.get("STACK_DBG", "0"))     # timeline of an A/B variant (exact ones: 16, 32)
for _ in range(20):
    fn(s)
torch.cuda.synchronize()
raw = ts.view(nblk, nw, 32).cpu().numpy().astype(np.float64)
t = raw[:, :, :16] * 0.01   # 100 MHz -> us
clk = raw[:, :, 16:]
last_i = 1 + 4 * a.n
mhz = (clk[:, :, last_i] - clk[:, :, 0]) / np.maximum(t[:, :, last_i] - t[:, :, 0], 1e-9)
print("shader clock during the kernel: median %.0f MHz (min %.0f, max %.0f)" % (np.median(mhz), mhz.min(), mhz.max()))
a.ts = 0
t0 = t[:, :, 0].min()
t = t - t0
names = ["start", "staged"]
for l in range(a.n):
    names += ["L%d zero+tab" % l, "L%d tiles(w)" % l, "L%d barrier" % l, "L%d stored" % l]
starts = t[:, 0, 0]
print("workgroup start: median %.2f  p90 %.2f  max %.2f us" % (np.median(starts), np.percentile(starts, 90),
                                                                starts.max()))
print("%-16s %8s %8s %8s   (us since first wave start; per-wave)" % ("phase end", "median", "p90", "max"))
prev = None
for i, nm in enumerate(names):
    v = t[:, :, i].reshape(-1)
    rel = (t[:, :, i] - t[:, :, 0]).reshape(-1)
    print("%-16s %8.2f %8.2f %8.2f   since own start: median %.2f" % (nm, np.median(v), np.percentile(v, 90),
                                                                    v.max(), np.median(rel)))
last = 1 + 4 * a.n
end = t[:, :, last]
print("kernel span (first start -> last wave done): %.2f us" % end.max())
# per-phase durations per wave (median)
print("phase durations (median over waves, us):")
for i in range(1, last + 1):
    dur = (t[:, :, i] - t[:, :, i - 1]).reshape(-1)
    print("  %-16s %7.2f  (p90 %.2f)" % (names[i], np.median(dur), np.percentile(dur, 90)))

d14 = (t[:, :, 14] - t[:, :, 2 + 4 * (a.n - 1)]).reshape(-1)
d15 = (t[:, :, 15] - t[:, :, 14]).reshape(-1)
print("last layer, first tile: k-loop done %.2f us after the layer barrier (median; p90 %.2f), epilogue %.2f (p90 %.2f)"
      % (np.median(d14), np.percentile(d14, 90), np.median(d15), np.percentile(d15, 90)))

# A/B: row-aligned layer path (dbg 0) vs generic layer path (dbg 16), interleaved rounds
def _t(reps=40):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn(s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


a.dbg = 0
res = {0: [], 16: [], 32: []}
for _ in range(5):
    for dbg in (0, 16, 32):
        a.dbg = dbg
        _t(5)
        res[dbg].append(_t())
a.dbg = 0
print("A/B conv_stack_fwd us: rows path %.2f (min %.2f) | generic %.2f (min %.2f) | no weight prefetch %.2f (min %.2f)"
      % (np.median(res[0]), min(res[0]), np.median(res[16]), min(res[16]), np.median(res[32]), min(res[32])))
