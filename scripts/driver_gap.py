"""Why does the driver's short bench (--steps 20 --warmup 5) read slower than long runs?

Builds the bench model exactly as bench.py does, captures the same graphs (a 5-step warmup
graph and the 20-step timed graph), then times the 20-step replay REPEATEDLY in one process,
each one bracketed like bench.time_steps (barrier + synchronize on both sides), and prints
per-replay wall and HIP-event ms/step.  If replay 1 is slow and later replays are fast, the
gap is a warm-up effect of the process (which one: see the --idle-ms variant, an idle gap
before each replay, and the kernel trace of the same run); if every replay is slow, it is
the short graph itself.

    python scripts/driver_gap.py [--reps 30] [--steps 20] [--warmup 5] [--idle-ms 0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=32)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep before each timed replay")
    ap.add_argument("--spin-ms", type=float, default=0.0,
                    help="GPU busy-loop (replays of the warmup graph) for this long before the first timed replay")
    a = ap.parse_args()
    import torch
    import bench
    from cori_intml_examples_amd.parallel import hvd
    hvd.init()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("INTML_DEVICE", str(dev))

    class Args:
        model, channels, samples = "rpv", 3, 32768
    model, shape, ncls, *_ = bench.build(Args, 1, False, dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    data = bench.synthetic(Args.samples, shape, ncls, model._executor, dev, g)
    B = 128
    if a.spin_ms > 0:
        # the bench's own warmup first, then keep the GPU busy on the same kind of work
        bench.time_steps(model, data, B, a.warmup, 0, a.chunk, g, dev)
        t_end = time.perf_counter() + a.spin_ms / 1e3
        while time.perf_counter() < t_end:
            bench.time_steps(model, data, B, a.warmup, 0, a.chunk, g, dev)
    rows = []
    for i in range(a.reps):
        if a.idle_ms > 0:
            time.sleep(a.idle_ms / 1e3)
        # rep 0 = exactly the bench's time_steps (warmup + one untimed replay of the timed graph)
        e, per = bench.time_steps(model, data, B, a.steps, a.warmup if i == 0 else 0, a.chunk, g, dev)
        rows.append((i, e / a.steps * 1e3, per[0] if per else None))
        print("rep %2d wall %.4f ms/step  event %.4f ms/step" % rows[-1], flush=True)
    print(json.dumps({"steps": a.steps, "warmup": a.warmup, "idle_ms": a.idle_ms, "spin_ms": a.spin_ms,
                      "first_wall": rows[0][1], "rest_wall_median": sorted(r[1] for r in rows[1:])[len(rows[1:]) // 2]
                      if len(rows) > 1 else None}))


if __name__ == "__main__":
    main()
