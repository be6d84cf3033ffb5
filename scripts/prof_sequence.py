"""Per-launch durations of ONE training step, in launch order, from a rocprofv3 kernel trace
(--kernel-trace --output-format csv: run_kernel_trace.csv).  The step is found as the
stretch between two consecutive launches of an anchor kernel that runs once per step (default
the head kernel); the median duration of each position over the last N steps is printed, so
kernels that run several times per step (the legacy model's three wgrad_gl launches) show
per layer.

    python scripts/prof_sequence.py run_kernel_trace.csv [anchor] [steps]
"""
import csv
import statistics
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "head_kernel"
nlast = int(sys.argv[3]) if len(sys.argv) > 3 else 10
rows = list(csv.DictReader(open(path)))
key_s = "Start_Timestamp" if "Start_Timestamp" in rows[0] else "Start_Timestamp_ns"
key_e = "End_Timestamp" if "End_Timestamp" in rows[0] else "End_Timestamp_ns"
rows.sort(key=lambda r: int(r[key_s]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
steps = [rows[a:b] for a, b in zip(idx[:-1], idx[1:])][-nlast:]
if not steps:
    sys.exit("no complete step found for anchor %r" % anchor)
n = min(len(s) for s in steps)
print("%3s %-70s %9s %9s" % ("#", "kernel (launch order from the anchor)", "med_us", "gap_us"))
tot = 0.0
for j in range(n):
    d = [(int(s[j][key_e]) - int(s[j][key_s])) / 1e3 for s in steps]
    gaps = [(int(s[j][key_s]) - int(s[j - 1][key_e])) / 1e3 for s in steps] if j else [0.0]
    md = statistics.median(d)
    tot += md
    print("%3d %-70s %9.2f %9.2f" % (j, steps[0][j]["Kernel_Name"][:70], md, statistics.median(gaps)))
print("step: %d launches, kernel sum %.1f us (median over the last %d steps)" % (n, tot, len(steps)))
