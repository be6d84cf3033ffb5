"""Worker for tests/test_dp.py::test_plane_choice_is_rank0s (gloo, CPU): the data plane an
``auto`` job runs must be ONE plane for every rank -- rank 0's choice is broadcast by
NativeGradReducer.configure, so a verdict file that only some ranks see (written between their
reads, or a per-rank cache directory) cannot split the job between planes."""
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cori_intml_examples_amd.parallel import dist as D  # noqa: E402


def main(out_dir, scenario):
    rank = int(os.environ["RANK"])
    # rank 1 (or rank 0) alone has a measured xGMI verdict for this job's key
    os.environ["INTML_PLANE_VERDICTS"] = os.path.join(out_dir, "verdicts%d.json" % rank)
    holder = 1 if scenario == "rank1" else 0
    D.init()
    grad_bytes = 4 * 547841
    if rank == holder:
        D.record_verdict(D.size(), grad_bytes, "xgmi")
    D.torch.cuda.is_available = lambda: True          # a GPU per rank on one node
    D.torch.cuda.device_count = lambda: 2
    red = object.__new__(D.NativeGradReducer)
    red.store = types.SimpleNamespace(numel=547841)
    red.comm = object()                               # an RCCL communicator (not used here)
    red.rank, red.size, red.compression, red.bucket_bytes = rank, 2, None, None
    red.buckets, red.bucket_groups, red._stage, red._configured = [(0, 547841)], [[0]], {}, False
    red.xgmi, red.xgmi_bucket = None, None
    red._setup_xgmi = lambda: None
    red.configure([(23584, 547841), (0, 23584)])
    rep = {"rank": rank, "local_view": D.auto_plane(grad_bytes), "plane": red.plane}
    with open(os.path.join(out_dir, "vote%d.json" % rank), "w") as f:
        json.dump(rep, f)
    D.shutdown()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
