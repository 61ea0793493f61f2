"""HBM traffic of the Schur-assembly kernels from rocprofv3 PMC passes.

Usage (on the GPU box, each counter in its own pass as MI355X_MICROARCH.md prescribes):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/f -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/w -o run -- python3 bench.py ...
    python3 tools/pmc_traffic.py gpurun_out/pmc/f/run_counter_collection.csv \
        gpurun_out/pmc/w/run_counter_collection.csv profiles/r01_schur_pmc.json

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  The Schur stage is schur_fused_f64 alone
(round 3: V^T X^-1 and V^T Y formed on chip); with CLRSDP_SCHUR_FUSED_Y=0 also the TYt GEMM
(gemm_f64_uni / gemm_f64_lds <false, true, 3, ...>, TAG 3, ahead on the side stream), and with
CLRSDP_SCHUR_FUSED=0 the TXt GEMM (TAG 1), the TYt GEMM and schur_pairs_f64.  Reported:
the per-launch mean of each and their sum per iteration, in bytes.  gfx950 correction: the guide
measured FETCH_SIZE = 1/2 of the bytes for 16-B-per-lane streaming reads; these kernels read
8 B per lane (global_load_dwordx2), a width the guide calls uncalibrated, so the raw counter and
the x2-corrected value are both written and `traffic` uses the raw value (the lower bound).
"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = {"tx": ("gemm_f64_", "<false, true, 1,"), "ty": ("gemm_f64_", "<false, true, 3,"),
           "pairs": ("schur_pairs_f64",), "fused": ("schur_fused_f64",)}


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for k, pat in KERNELS.items():
            if all(x in r["Kernel_Name"] for x in pat):
                vals[k].append(float(r["Counter_Value"]) * 1024.0)  # KB -> B
    return {k: sum(v) / len(v) for k, v in vals.items() if v}, {k: len(v) for k, v in vals.items()}


def main():
    fpath, wpath, out = sys.argv[1:4]
    fetch, nf = per_kernel(fpath, "FETCH_SIZE")
    write, nw = per_kernel(wpath, "WRITE_SIZE")
    res = {
        "kernels": {k: {"fetch_bytes": fetch.get(k), "fetch_bytes_x2": 2 * fetch.get(k, 0.0),
                        "write_bytes": write.get(k), "dispatches": nf.get(k)} for k in KERNELS},
    }
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _clrsdp_pkg
    res["source_hash"] = _clrsdp_pkg.load_build().source_hash()   # the build the counters saw
    res["traffic_bytes_per_iteration"] = sum(fetch.values()) + sum(write.values())
    res["traffic_bytes_per_iteration_fetch_x2"] = 2 * sum(fetch.values()) + sum(write.values())
    res["note"] = ("FETCH_SIZE at 8 B/lane is uncalibrated on gfx950 (MI355X_MICROARCH.md §HBM); "
                   "traffic uses the raw counter, fetch_x2 is the 16-B-calibrated upper reading")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
