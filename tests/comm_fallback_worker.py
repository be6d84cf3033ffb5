"""CPU worker for tests/test_dp.py::test_rccl_init_failure_falls_back_collectively: every rank's
RCCL communicator construction is made to fail (as on a node whose RCCL cannot come up) and
dist.init must vote the whole job onto the RCCL-free plane -- no rank raises, no rank hangs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cori_intml_examples_amd.parallel import comm as C  # noqa: E402
from cori_intml_examples_amd.parallel import dist  # noqa: E402


class _Broken:
    def __init__(self, *a, **k):
        raise RuntimeError("ncclCommInitRank: unhandled system error (injected)")


def main(outdir):
    C.comm_mode = lambda *a, **k: "native"      # what a multi-GPU node selects
    C.NativeComm = _Broken
    st = dist.init()
    rep = {"rank": st.rank, "size": st.size, "xgmi_only": bool(st.xgmi_only), "comm": st.comm is not None}
    with open(os.path.join(outdir, "fb%d.json" % st.rank), "w") as f:
        json.dump(rep, f)
    dist.shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
