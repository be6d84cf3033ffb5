"""Summarise a rocprofv3 kernel_stats.csv: per-kernel avg time and per-step totals.

    python scripts/prof_summary.py run_kernel_stats.csv [anchor-substring]

The trace covers warmup, graph capture and the timed steps, so a kernel's call count is
not a multiple of the timed steps.  Per-step cost is therefore avg_us x launches-per-step,
where launches-per-step = round(calls / anchor calls) and the anchor is a kernel that runs
exactly once per training step (default: the head kernel; the prologue-free step has no
prologue launch).  Kernels that run fewer
times than the anchor (setup, data generation) are listed but not summed.
"""
import csv
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].isdigit() else "head_kernel"
rows = list(csv.DictReader(open(path)))
anchor_calls = max((int(r["Calls"]) for r in rows if anchor in r["Name"]), default=0)
if anchor_calls == 0:
    anchor_calls = max(int(r["Calls"]) for r in rows)
tot = 0.0
print("%-62s %7s %10s %9s %9s" % ("kernel", "calls", "avg_us", "per_step", "us/step"))
for r in rows:
    calls = int(r["Calls"])
    avg = float(r["AverageNs"]) / 1e3
    per_step = round(calls / anchor_calls) if calls >= anchor_calls * 0.9 else 0
    per = avg * per_step
    tot += per
    print("%-62s %7d %10.2f %9d %9.2f" % (r["Name"][:62], calls, avg, per_step, per))
print("sum of per-step kernels (avg x launches/step, anchor %s x%d): %.1f us"
      % (anchor, anchor_calls, tot))
