"""Per-iteration busy time and idle gaps from a rocprofv3 kernel trace: iterations are split at
each eigmin launch (one per loop body); prints the span, the summed kernel-busy time (union of
intervals) and the largest idle gaps of the last few iterations."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "eigmin" in r["Kernel_Name"]]
for a, b in zip(idx[-6:-1], idx[-5:]):
    seg = rows[a + 1:b + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, r["Kernel_Name"][:40]))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    gaps.sort(reverse=True)
    print("span %.1f us  busy %.1f us  kernels %d  idle %.1f us  largest gaps: %s" % (
        (t1 - t0) / 1e3, busy / 1e3, len(seg), (t1 - t0 - busy) / 1e3,
        ", ".join("%.1f (before %s)" % (g / 1e3, n) for g, n in gaps[:4])))
