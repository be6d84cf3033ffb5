"""Per-launch A/B of INTML_TUNE variants on the RPV (or MNIST) bench step.

    python scripts/ab_launches.py "lds_layout=0" "lds_layout=1" [--model mnist] [--batch 128]

Builds one model per variant (the tune switches are read when the step's launch list is
built), runs one real step so buffers hold realistic data, then times every launch alone
(HIP events, 40 reps) in interleaved rounds (variant A, B, A, B, ...) and prints the median
per launch and the sum, so same-box noise hits every variant alike.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

os.environ["INTML_GRAPHS"] = "0"


def build(model, B, dev):
    from cori_intml_examples_amd.apps import zoo
    if model == "legacy":
        m = zoo.rpv_legacy_cnn((64, 64, 1), device=dev)
        shape = (64, 64, 1)
        rs = np.random.RandomState(0)
        y = (rs.rand(B * 4) > 0.5).astype(np.float32)
    elif model == "mnist":
        m = zoo.mnist_cnn(32, 64, 128, 0.25, 0.5, lr=1.0, device=dev)
        shape = (28, 28, 1)
        rs = np.random.RandomState(0)
        y = np.eye(10, dtype=np.float32)[rs.randint(0, 10, B * 4)]
    else:
        m = zoo.rpv_cnn((64, 64, 3), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2, optimizer="Adam",
                        lr=1e-3, device=dev)
        shape = (64, 64, 3)
        rs = np.random.RandomState(0)
        y = (rs.rand(B * 4) > 0.5).astype(np.float32)
    x = rs.rand(B * 4, *shape).astype(np.float32)
    ex = m._executor
    ex.use_graphs = False
    d = ex.upload(x, y)
    ex.train_step(d, torch.arange(d.n, device=dev), 0, B)
    torch.cuda.synchronize()
    return m, ex._plans[(B, "train")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--model", default="rpv")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    plans = []
    for v in a.variants:
        os.environ["INTML_TUNE"] = v
        plans.append(build(a.model, a.batch, dev))
    os.environ.pop("INTML_TUNE", None)
    s = torch.cuda.current_stream().cuda_stream

    def timeit(fn, reps=40):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            fn(s)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn(s)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    res = [{} for _ in plans]
    for _ in range(a.rounds):
        for i, (_, bp) in enumerate(plans):
            for it in bp.launches:
                res[i].setdefault(it[0], []).append(timeit(it[1]))
    names = []
    for r in res:
        for k in r:
            if k not in names:
                names.append(k)
    print("%-26s " % "launch" + " ".join("%22s" % v[:22] for v in a.variants))
    tot = [0.0] * len(plans)
    for n in names:
        row = []
        for i, r in enumerate(res):
            if n in r:
                m = float(np.median(r[n]))
                tot[i] += m
                row.append("%22.2f" % m)
            else:
                row.append("%22s" % "-")
        print("%-26s " % n + " ".join(row))
    print("%-26s " % "SUM (launches alone)" + " ".join("%22.2f" % t for t in tot))


if __name__ == "__main__":
    main()
