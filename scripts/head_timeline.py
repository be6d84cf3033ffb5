"""Phase stamps of the head kernel (fused dense epilogue + loss + backward) for the RPV B=128 step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cori_intml_examples_amd.apps import zoo

os.environ["INTML_GRAPHS"] = "0"
dev = torch.device("cuda", 0)
B = 128
rs = np.random.RandomState(0)
if os.environ.get("MODEL", "rpv") == "mnist":
    model = zoo.mnist_cnn(32, 64, 128, 0.25, 0.5, lr=1.0, device=dev)
    ex = model._executor
    ex.use_graphs = False
    d = ex.upload(rs.rand(B * 4, 28, 28, 1).astype(np.float32), np.eye(10, dtype=np.float32)[rs.randint(0, 10, B * 4)])
else:
    model = zoo.rpv_cnn((64, 64, 3), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2, optimizer="Adam",
                        lr=1e-3, device=dev)
    ex = model._executor
    ex.use_graphs = False
    d = ex.upload(rs.rand(B * 4, 64, 64, 3).astype(np.float32), (rs.rand(B * 4) > 0.5).astype(np.float32))
ex.train_step(d, torch.arange(d.n, device=dev), 0, B)
torch.cuda.synchronize()
bp = ex._plans[(B, "train")]
s = torch.cuda.current_stream().cuda_stream
fn = [f for (n, f, *_) in bp.launches if n == "head"][0]
a = fn.__defaults__[0]
ts = torch.zeros(B * 8, dtype=torch.int64, device=dev)
a.ts = ts.data_ptr()
for _ in range(10):
    fn(s)
torch.cuda.synchronize()
a.ts = 0
t = ts.view(-1, 8).cpu().numpy().astype(np.float64) * 0.01
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
print("head: %d blocks, start spread med %.2f max %.2f us, span %.2f us" % (
    len(t), np.median(t[:, 0] - t0), (t[:, 0] - t0).max(), (t[:, 6] - t0).max()))
print("  dot+shuffles       +%.2f us (median, inside dot+loss)" % np.median(t[:, 7] - t[:, 1]))
for i, lab in enumerate(["epilogue+w stage", "dot+loss", "barrier", "metrics atomics", "dW slab", "bwd-through"]):
    print("  %-18s +%.2f us (median)" % (lab, np.median(t[:, i + 1] - t[:, i])))
