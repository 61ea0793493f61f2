"""Dump one loop body from a rocprofv3 kernel trace in launch order: start offset, duration, queue
and kernel name (iterations split at each eigmin launch, as in iter_gaps.py)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "eigmin" in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
seg = rows[a + 1:b + 1]
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f %7.1f q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, r.get("Queue_Id", "?"),
                                     r["Kernel_Name"][:90]))
