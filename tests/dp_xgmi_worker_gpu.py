"""GPU worker for tests/test_comm.py::test_dp_step_xgmi_ranks_one_gpu: the 8-GPU data-parallel
training step, rehearsed with P ranks on ONE MI355X.

RCCL refuses two ranks on one GPU; the RCCL-free data plane (``INTML_COMM=xgmi``, chosen on
its own when ranks share a GPU) is the same fused xGMI all-reduce + Adam kernel, captured into
the same HIP graph, that an 8-GPU job uses -- only the peers' inboxes live on this card.

Every rank trains the RPV bench model (conv [16,32,64], fc [128], dropout 0 so the rows of a
global batch see the same masks wherever they run) for 24 steps as 3 graph replays of 8
captured steps, per-rank batch 128/P: global step t uses rows perm[128t : 128t+128] of one
device-resident synthetic data set, rank r rows perm[128t + r*128/P : ...].  Rank 0 then
trains a single-process model from the same initial weights on the same permutation at
batch 128.  Writes one JSON per rank:
  err            the fused kernel's error word (0: no wait timed out)
  digest         sha256 of the rank's trained fp32 weights (all ranks must agree bitwise)
  vs_single      rank 0: p999 / max |w_dp - w_single|
for Adam (the production optimizer, fused into the xGMI kernel) and SGD (linear update: the
DP-vs-single bound is tight).
"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from cori_intml_examples_amd.apps import zoo  # noqa: E402
from cori_intml_examples_amd.io import synth  # noqa: E402
from cori_intml_examples_amd.parallel import dist, hvd  # noqa: E402
from cori_intml_examples_amd.utils import set_random_seed  # noqa: E402

GLOBAL_B, STEPS, SPG, N = 128, 24, 8, 4096
# DPX_SMALL=1: a small RPV-shaped model (32x32x3, conv [8,16,16], fc [32]) whose exchange tables
# have a handful of blocks -- small enough that the separate-GPU geometry (one workgroup per
# table block, INTML_TUNE=xgmi_xchg_wg=0) cannot fill the shared card with spinning workgroups
SMALL = os.environ.get("DPX_SMALL", "0") == "1"
SHAPE = (32, 32, 3) if SMALL else (64, 64, 3)
ARCH = dict(conv_sizes=[8, 16, 16], fc_sizes=[32]) if SMALL else dict(conv_sizes=[16, 32, 64], fc_sizes=[128])


def flat(m):
    return np.concatenate([w.reshape(-1) for w in m.get_weights()])


def train(m, data, perm, bs):
    ex = m._executor
    for i in range(STEPS // SPG):
        ex.train_steps(data, perm, i * SPG * bs, bs, SPG)
    torch.cuda.synchronize()
    return flat(m)


def run(opt, lr, outdir, r, P, dev):
    """One DP training of the bench model with `opt`; rank 0 also trains the single-process
    twin.  Returns this rank's report."""
    rep = {}
    kw = dict(dropout=0.0, optimizer=opt, lr=lr, device="cuda:0", **ARCH)
    set_random_seed(1 + r)                       # different on purpose: the broadcast must fix it
    m = zoo.rpv_cnn(SHAPE, use_horovod=True, **kw)
    hvd.broadcast_global_variables(0, model=m)
    w0 = m.get_weights()
    ex = m._executor
    data = synth.synth_device("rpv", N, SHAPE, 1, ex.in_Cs, 7, dev)
    g = torch.Generator(device=dev).manual_seed(11)
    perm = torch.randperm(N, device=dev, generator=g)[:STEPS * GLOBAL_B]
    b = GLOBAL_B // P
    mine = perm.view(STEPS, P, b)[:, r, :].reshape(-1).contiguous()
    red = ex.reducer
    try:
        w = train(m, data, mine, b)
        red.after_step()                         # raises if an earlier launch's wait timed out
    except Exception as e:                       # diagnostics for the test's failure message
        plan = next(iter(ex._plans.values()), None)
        x = red.xgmi
        rep.update(error=str(e), err=x.err.tolist() if x is not None else None,
                   ctr=x.ctr[:x.grid].tolist() if x is not None else None,
                   launches=[it[0] for it in plan.launches] if plan is not None else None)
        with open(os.path.join(outdir, "dpx%d.json" % r), "w") as f:
            json.dump({opt: rep}, f, indent=1)
        raise
    plan = next(iter(ex._plans.values()))
    rep["reducer"] = type(red).__name__
    rep["plane"] = red.plane
    rep["buckets"] = [list(x) for x in red.buckets]
    rep["comm_in_graph"] = bool(plan.comm_in_graph)
    rep["fused_launches"] = [it[0] for it in plan.launches if "xgmi" in it[0] or "allreduce" in it[0]]
    # producer push: the launches that reduce the early (head / dense) groups inside the
    # backward and push them to their owners' inboxes, and the range the all-reduce skips
    rep["push_launches"] = sorted((getattr(plan, "early_push", None) or {}).keys())
    rep["pushed"] = list(getattr(plan, "pushed", None) or [])
    rep["xchg_launches"] = sorted((getattr(plan, "early_xchg", None) or {}).keys())
    rep["exchanged"] = bool(getattr(plan, "exchanged", False))
    rep["xchg_fin"] = getattr(plan, "xchg_fin", None) is not None     # split exchange: finish half at the end
    rep["bucket_xchg"] = sorted((getattr(plan, "bucket_xchg", None) or {}).keys())
    # exchange geometry: looping workgroups (nx > 0, ranks sharing a GPU) or one per block (0)
    rep["xchg_nx"] = sorted({int(v[1].nx) for v in (getattr(plan, "early_xchg", None) or {}).values()}
                            | {int(v.nx) for v in (getattr(plan, "bucket_xchg", None) or {}).values()})
    rep["shared"] = bool(red.xgmi.shared) if red.xgmi is not None else None
    rep["err"] = int(red.xgmi.err[0].item()) if red.xgmi is not None else -1
    rep["digest"] = hashlib.sha256(w.tobytes()).hexdigest()
    rep["finite"] = bool(np.isfinite(w).all())
    rep["moved"] = float(np.abs(w - np.concatenate([a.reshape(-1) for a in w0])).max())
    if r == 0:
        single = zoo.rpv_cnn(SHAPE, use_horovod=False, **kw)
        single.set_weights(w0)
        ws = train(single, data, perm.contiguous(), GLOBAL_B)
        d = np.abs(w - ws)
        step = float(np.linalg.norm(ws - np.concatenate([a.reshape(-1) for a in w0])))
        rep["vs_single"] = {"p999": float(np.quantile(d, 0.999)), "max": float(d.max()), "step_norm": step,
                            "rel": float(np.linalg.norm(w - ws) / max(step, 1e-30))}
    return rep


def main(outdir):
    st = hvd.init()
    r, P = hvd.rank(), hvd.size()
    dev = torch.device("cuda", 0)
    out = {"rank": r, "size": P, "xgmi_only": bool(st.xgmi_only), "rccl": st.comm is not None}
    # Adam: the production optimizer (fused into the xGMI kernel); SGD: its update is linear in
    # the gradient, so the DP-vs-single difference stays at the all-reduce's reordering level
    # (Adam turns a last-ulp difference of a near-zero gradient into up to a full lr step)
    out["Adam"] = run("Adam", 1e-3, outdir, r, P, dev)
    out["SGD"] = run("SGD", 0.05, outdir, r, P, dev)
    hvd.barrier()
    with open(os.path.join(outdir, "dpx%d.json" % r), "w") as f:
        json.dump(out, f, indent=1)
    dist.shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
