"""Print the kernel timeline of the last few training steps from a rocprofv3 kernel_trace.csv
(start offset, duration, queue/stream), to see overlap and gaps between launches."""
import csv
import sys

path = sys.argv[1]
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-nlast:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print("%9.2f %8.2f gap%7.2f q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r.get("Queue_Id", r.get("Stream_Id", "?")),
                                            r["Kernel_Name"][:70]))
    prev_end = e if prev_end is None else max(prev_end, e)
