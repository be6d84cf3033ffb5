"""Summarise a rocprofv3 kernel_stats.csv: per-kernel avg time and per-step totals."""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
tot = 0.0
print("%-62s %7s %10s %9s" % ("kernel", "calls", "avg_us", "us/step"))
for r in rows:
    calls = int(r["Calls"])
    avg = float(r["AverageNs"]) / 1e3
    per = float(r["TotalDurationNs"]) / 1e3 / steps
    if calls >= steps:
        tot += per
    print("%-62s %7d %10.2f %9.2f" % (r["Name"][:62], calls, avg, per))
print("sum of per-step kernels (calls >= steps): %.1f us" % tot)
