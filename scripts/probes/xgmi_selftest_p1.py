"""Run the xGMI plane's admission self-test at one rank (size 1) and print what it reports."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from cori_intml_examples_amd.parallel import xgmi as X  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for n in (547841, 100003):
    x = X.XgmiAllreduce(0, 1, n, dev, lambda v: [v])
    print("n", n, "setup", x.setup_error, flush=True)
    x.args.timeout_ticks = 5 * X._TICKS_PER_S
    print("selftest(stress 0)", x.selftest(stress=0), flush=True)
    print("selftest(default)", x.selftest(), flush=True)
    print("err", x.err.tolist(), flush=True)
    x.close()
