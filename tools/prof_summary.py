"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel total/avg and per-iteration share.

The runtime's copy and fill kernels (__amd_rocclr_copyBuffer / fillBuffer*) are listed apart and
left out of the per-iteration sum: most of them are set-up work outside the loop (instance upload,
plan descriptors, state snapshots of bench.py); inside the loop each body carries exactly one
copy, the ~1 KB stats read-back (tools/copy_census.py)."""
import csv
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
# loop bodies: the eigen-solver launches (one per body; eigmin_mx's flagged eigmin_lds2 launch
# is its second and is not counted when eigmin_mx ran)
iters = float(sys.argv[2]) if len(sys.argv) > 2 else \
    float(sum(int(r["Calls"]) for r in rows if "eigmin" in r["Name"] and
              "eigmin_lds2" not in r["Name"]) or
          sum(int(r["Calls"]) for r in rows if "eigmin" in r["Name"]) or 1)
lib = [r for r in rows if not r["Name"].startswith("__amd_rocclr")]
rt = [r for r in rows if r["Name"].startswith("__amd_rocclr")]
tot = sum(float(r["TotalDurationNs"]) for r in lib)
print("%-64s %6s %10s %9s %9s %6s" % ("kernel", "calls", "total_us", "avg_us", "us/iter", "%"))
for r in lib[:40]:
    t = float(r["TotalDurationNs"]) / 1e3
    print("%-64s %6s %10.1f %9.2f %9.1f %6.2f" % (r["Name"][:64], r["Calls"], t, float(r["AverageNs"]) / 1e3, t / iters, float(r["Percentage"])))
print("sum of library kernel time per iteration: %.1f us (%d loop bodies)" % (tot / 1e3 / iters, iters))
if rt:
    print("runtime copies / fills (mostly set-up outside the loop; one stats copy per body inside it):")
    for r in rt:
        print("  %-62s %6s %10.1f us total %9.2f avg" % (r["Name"][:62], r["Calls"],
                                                        float(r["TotalDurationNs"]) / 1e3,
                                                        float(r["AverageNs"]) / 1e3))
