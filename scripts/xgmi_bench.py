"""Microbenchmark of the fused xGMI all-reduce kernel at one rank (local uncached memory):
us per launch, sum-only and with the fused Adam update, for a few gradient sizes."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cori_intml_examples_amd.parallel import xgmi as X
from cori_intml_examples_amd.ops.hip import kernels

K = kernels()
dev = torch.device("cuda", 0)
for n in [int(v) for v in os.environ.get("XG_SIZES", "548129,1096258,4385032").split(",")]:
    x = X.XgmiAllreduce(0, 1, n, dev, lambda o: [o])
    g = torch.randn(n, device=dev)
    p = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    st = torch.zeros(K.STEP_STATE_BYTES, dtype=torch.uint8, device=dev)
    a = K.OptimArgs()
    a.p, a.g, a.s0, a.s1, a.n, a.st, a.kind = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, st.data_ptr(), 3
    s = torch.cuda.current_stream().cuda_stream
    for mode in (0, 1):
        for _ in range(10):
            x.launch(g.data_ptr(), s, opt=a if mode else None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            x.launch(g.data_ptr(), s, opt=a if mode else None)
        e1.record()
        torch.cuda.synchronize()
        print("n=%d grid=%d mode=%d: %.2f us/launch (err=%d)" % (n, x.grid, mode, e0.elapsed_time(e1) / 200 * 1e3,
                                                             int(x.err.item())), flush=True)
    c = torch.empty_like(g)
    e0.record()
    for _ in range(200):
        c.copy_(g)
    e1.record()
    torch.cuda.synchronize()
    print("   plain device copy of the gradient: %.2f us" % (e0.elapsed_time(e1) / 200 * 1e3))
    x.close()
