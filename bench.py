#!/usr/bin/env python
"""Headline benchmark: RPV CNN training throughput (images/sec, whole job).

BASELINE.json metric "images/sec (whole node) RPV CNN at 1/2/4/8 MI355X"; config
"ATLAS RPV 3-channel calorimeter-image CNN data-parallel bf16 (DistTrain_rpv)":
conv [16,32,64] 3x3 'same' + ReLU + 2x2 max-pool, Dropout(0.2), Dense(128)+ReLU,
Dropout(0.2), Dense(1)+sigmoid, binary cross-entropy, Adam(lr = 0.001 * size),
batch 128 per rank (DistTrain_rpv.ipynb:267-285), 64x64x3 input.

Each timed step is a FULL training step: device-side batch gather from the resident
(synthetic) dataset by the epoch permutation, forward, loss, backward, bucketed RCCL
gradient all-reduce (N > 1), Adam update + weight re-pack.  Weak scaling: per-GPU batch
fixed.  Launch: ``python bench.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_IMG_PER_S = 1240.0   # RPV single-GPU reference, Train_rpv.ipynb:304-312
BASELINE_MNIST_IMG_PER_S = 43600.0   # MNIST DP aggregate, 8 Haswell nodes, DistTrain_mnist.ipynb:341-357


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=128, help="per-GPU batch (reference: 128)")
    ap.add_argument("--channels", type=int, default=3)
    ap.add_argument("--samples", type=int, default=32768, help="resident synthetic samples per rank")
    ap.add_argument("--model", default="rpv", choices=["rpv", "mnist", "rpv_legacy"])
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--steps-per-graph", type=int, default=int(os.environ.get("INTML_STEPS_PER_GRAPH", 8)),
                    help="full training steps per HIP-graph replay (the fit() loop's default)")
    args = ap.parse_args()
    if args.no_graphs:
        os.environ["INTML_GRAPHS"] = "0"

    import torch
    from cori_intml_examples_amd.parallel import hvd
    from cori_intml_examples_amd.apps import zoo
    from cori_intml_examples_amd.models.executor_base import DeviceData

    world = int(os.environ.get("WORLD_SIZE", "1"))
    hvd.init()
    rank, size = hvd.rank(), hvd.size()
    local = hvd.local_rank()
    torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
    dev = torch.device("cuda", torch.cuda.current_device())
    os.environ.setdefault("INTML_DEVICE", str(dev))

    B = args.batch
    # INTML_DP_FORCE=1 runs the full data-parallel step (RCCL all-reduces in the graph) at N=1
    dp = size > 1 or os.environ.get("INTML_DP_FORCE", "0") not in ("0", "")
    if args.model == "rpv":
        model = zoo.rpv_cnn((64, 64, args.channels), conv_sizes=[16, 32, 64], fc_sizes=[128], dropout=0.2,
                            optimizer="Adam", lr=0.001 * size, use_horovod=dp, device=dev)
        shape, ncls = (64, 64, args.channels), 1
        cfg_name = "RPV CNN conv[16,32,64] fc[128] 64x64x%d (DistTrain_rpv)" % args.channels
        metric, baseline = "images/sec (whole node) RPV CNN training", BASELINE_IMG_PER_S
    elif args.model == "mnist":
        model = zoo.mnist_cnn(32, 64, 128, 0.25, 0.5, lr=1.0 * size, use_horovod=dp, device=dev)
        shape, ncls = (28, 28, 1), 10
        cfg_name = "MNIST CNN 32-64-128 (DistTrain_mnist)"
        metric, baseline = "images/sec (whole node) MNIST CNN training", BASELINE_MNIST_IMG_PER_S
    else:
        model = zoo.rpv_legacy_cnn((64, 64, args.channels), device=dev, use_horovod=dp)
        shape, ncls = (64, 64, args.channels), 1
        cfg_name = "RPV legacy CNN 34.5M (Train_rpv)"
        metric, baseline = "images/sec (whole node) RPV legacy CNN training", BASELINE_IMG_PER_S

    ex = model._executor
    # synthetic, device-resident dataset (no network / files here)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    n = max(args.samples, B * 4)
    x = torch.rand((n,) + shape, generator=g, device=dev)
    xs = torch.zeros(n, shape[0], shape[1], ex.in_Cs, dtype=torch.bfloat16, device=dev)
    xs[..., :shape[2]] = x.to(torch.bfloat16)
    del x
    if ncls == 1:
        y = (torch.rand(n, 1, generator=g, device=dev) > 0.5).float()
    else:
        y = torch.nn.functional.one_hot(torch.randint(0, ncls, (n,), generator=g, device=dev), ncls).float()
    data = DeviceData(xs.reshape(n, -1), y, n)
    hvd.broadcast_global_variables(0, model=model)

    state = {"pos": 0, "perm": torch.randperm(n, device=dev, generator=g)}
    chunk = max(1, args.steps_per_graph)

    def run(k):
        """k full training steps; a run of steps is one HIP-graph replay (the step's
        bookkeeping is device-resident), re-shuffling when the epoch is exhausted."""
        if state["pos"] + k * B > n:
            state["pos"] = 0
            state["perm"] = torch.randperm(n, device=dev, generator=g)
        ex.train_steps(data, state["perm"], state["pos"], B, k)
        state["pos"] += k * B

    def chunks(total):
        return [chunk] * (total // chunk) + ([total % chunk] if total % chunk else [])

    ex.reset_metrics()
    timed = chunks(args.steps)
    for k in chunks(args.warmup) + sorted(set(timed)):   # every timed graph is captured here
        run(k)
    hvd.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in timed:
        run(k)
    torch.cuda.synchronize()
    hvd.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if size > 1:
        elapsed = max(hvd.allgather(elapsed))   # MAX over ranks
    loss, acc, cnt = ex.read_metrics()
    ms = elapsed / args.steps * 1e3
    value = size * B * args.steps / elapsed
    if rank == 0:
        out = {"metric": metric,
               "value": round(value, 1), "unit": "images/s", "n_gpus": size, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": round(value / baseline, 2),
               "dtype": "bf16", "data": "synthetic (device-resident, random-init weights)",
               "config": {"model": cfg_name, "global_batch": B * size, "per_gpu_batch": B,
                          "seq_len": None, "input": list(shape),
                          "optimizer": type(getattr(model.optimizer, "_base_optimizer", model.optimizer)).__name__,
                          "parallelism": "dp%d" % size, "steps_per_graph": chunk,
                          "train_loss": round(loss, 5)}}
        print(json.dumps(out), flush=True)
    hvd.shutdown()


if __name__ == "__main__":
    main()
