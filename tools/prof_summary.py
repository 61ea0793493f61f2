"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel total/avg and per-iteration share."""
import csv, sys
path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
# loop bodies: the eigen-solver launches (one per body; eigmin_mx's flagged eigmin_lds2 launch
# is its second and is not counted when eigmin_mx ran)
iters = float(sys.argv[2]) if len(sys.argv) > 2 else \
    float(sum(int(r["Calls"]) for r in rows if "eigmin" in r["Name"] and
              "eigmin_lds2" not in r["Name"]) or
          sum(int(r["Calls"]) for r in rows if "eigmin" in r["Name"]) or 1)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("%-64s %6s %10s %9s %9s %6s" % ("kernel", "calls", "total_us", "avg_us", "us/iter", "%"))
for r in rows[:40]:
    t = float(r["TotalDurationNs"]) / 1e3
    print("%-64s %6s %10.1f %9.2f %9.1f %6.2f" % (r["Name"][:64], r["Calls"], t, float(r["AverageNs"]) / 1e3, t / iters, float(r["Percentage"])))
print("sum of kernel time per iteration: %.1f us (%d loop bodies)" % (tot / 1e3 / iters, iters))
