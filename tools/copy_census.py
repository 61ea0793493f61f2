"""Where the runtime's copy/fill kernels (__amd_rocclr_copyBuffer / fillBufferAligned) of a
rocprofv3 kernel trace come from: before the first loop body (uploads, allocations), inside
loop bodies (split at each eigmin launch), and their count per body."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
eig = [i for i, r in enumerate(rows) if "eigmin" in r["Kernel_Name"]]
first_body = min(i for i, r in enumerate(rows) if "clrsdp::" in r["Kernel_Name"])
per = collections.Counter()
bodies = collections.defaultdict(collections.Counter)
for i, r in enumerate(rows):
    k = r["Kernel_Name"]
    if "rocclr" not in k:
        continue
    name = "copy" if "copy" in k else "fill"
    if i < first_body:
        per["before the first library kernel: " + name] += 1
        continue
    nb = sum(1 for e in eig if e < i)   # loop bodies completed before this one
    bodies[nb][name] += 1
    per["after the first library kernel: " + name] += 1
for k, v in sorted(per.items()):
    print("%-50s %d" % (k, v))
print("per body index (bodies split at eigmin):")
for nb in sorted(bodies):
    print("  body %3d: %s" % (nb, dict(bodies[nb])))
