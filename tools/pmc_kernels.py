"""Per-kernel PMC evidence from rocprofv3 counter passes (SQ/GRBM counters, one pass each).

Usage (on the GPU box; tools/profile_round.sh runs it):

    rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES ... -d D -o run -- python3 bench.py ...
    python3 tools/pmc_kernels.py D/run_counter_collection.csv KT/run_kernel_stats.csv out.json [clusters]

For each kernel family of the fp64 loop body (the batched GEMMs, the strip chains, the Cholesky
inverse, the step-length eigen-solver, the Schur kernel) it reports per dispatch: the counters'
means, the fp64 MFMA flops the kernel issued (SQ_INSTS_VALU_MFMA_F64 x 2048: one
v_mfma_f64_16x16x4f64 is 16x16x4 multiply-adds), their rate over the kernel's mean duration from
the kernel trace of the same build, the fraction of the 78.6 TF fp64 matrix peak, the wave-cycle
split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES, disjoint) and the
LDS bank-conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).  Where the algorithmic flop
count of a launch is known from the C3 shape (64 clusters, 128 x 128 blocks) the fraction of peak
on algorithmic flops is reported too.
"""
import csv
import json
import os
import sys
from collections import defaultdict

PEAK_TF = 78.6
MFMA_F64_FLOPS = 2 * 16 * 16 * 4
# kernel family -> substrings that must all occur in the kernel name
FAMILIES = {
    "gemm_f64_uni": ("gemm_f64_uni",),
    "gemm_f64_lds": ("gemm_f64_lds",),
    "gemm_f64_dyn": ("gemm_f64_dyn",),
    "chain_f64 (Z, dY)": ("chain_f64<false, false, false>",),
    "chain_f64 (step, SYM)": ("chain_f64<true, true, false>",),
    "chain_f64 (U = Z V + rhs)": ("chain_f64<false, false, true>",),
    "chol_inv_tiles<128>": ("chol_inv_tiles<128>",),
    "eigmin_split": ("eigmin_split",),
    "eigmin_reg": ("eigmin_reg",),
    "schur_fused_f64": ("schur_fused_f64",),
}


def algorithmic_flops(fam, blocks=64, n=128):
    """Algorithmic fp64 flops of one launch at the C3 shape (per the reference's operation)."""
    if fam == "chol_inv_tiles<128>":
        # Cholesky n^3/3 + triangular inverse n^3/3 per block; the X/Y launch has 2*blocks,
        # S11 / S22' launches blocks (the mean over the launches of a body: 4 launches, 5*blocks)
        return 2.0 * n ** 3 / 3.0 * (5 * blocks / 4)
    if fam == "eigmin_split":
        return 4.0 * n ** 3 / 3.0 * 2 * blocks  # Householder tridiagonalisation of X and Y blocks
    if fam == "chain_f64 (Z, dY)":
        return 2 * 2.0 * n ** 3 * blocks       # two n^3 products per block
    if fam == "chain_f64 (step, SYM)":
        return 2 * 2.0 * n ** 3 * 2 * blocks   # L^-1 dM L^-T for the X and the Y blocks
    if fam == "chain_f64 (U = Z V + rhs)":
        K = 2 * n - 1
        return 2.0 * n * n * K * blocks
    return None


def main():
    cpath, kpath, out = sys.argv[1:4]
    blocks = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(cpath)):
        name = r["Kernel_Name"]
        for fam, pat in FAMILIES.items():
            if all(p in name for p in pat):
                vals[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = {}
    for r in csv.DictReader(open(kpath)):
        for fam, pat in FAMILIES.items():
            if all(p in r["Name"] for p in pat):
                c, t = dur.get(fam, (0, 0.0))
                dur[fam] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]))
    res = {"peak_tflops": PEAK_TF, "blocks": blocks, "kernels": {}}
    for fam, cnt in vals.items():
        m = {k: sum(v) / len(v) for k, v in cnt.items()}
        rec = {"counters_mean_per_dispatch": m, "dispatches": max(len(v) for v in cnt.values())}
        if fam in dur and dur[fam][0]:
            us = dur[fam][1] / dur[fam][0] / 1e3
            rec["mean_duration_us"] = us
            if "SQ_INSTS_VALU_MFMA_F64" in m:
                fl = m["SQ_INSTS_VALU_MFMA_F64"] * MFMA_F64_FLOPS
                rec["mfma_f64_flops_issued"] = fl
                rec["issued_tflops"] = fl / us / 1e6
                rec["issued_frac_of_peak"] = fl / us / 1e6 / PEAK_TF
            alg = algorithmic_flops(fam, blocks)
            if alg:
                rec["algorithmic_flops"] = alg
                rec["algorithmic_frac_of_peak"] = alg / us / 1e6 / PEAK_TF
            if "GRBM_GUI_ACTIVE" in m:
                rec["effective_clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            rec["wave_cycle_split"] = {k: m.get(k, 0.0) / wc for k in
                                       ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
        if m.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_bank_conflict_share"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
        res["kernels"][fam] = rec
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _clrsdp_pkg
    res["source_hash"] = _clrsdp_pkg.load_build().source_hash()
    res["note"] = ("SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_ANY count quad-cycles summed over "
                   "waves; the split is their ratio.  issued_frac_of_peak prices the MFMA "
                   "instructions the kernel executed (padding and symmetric halves included), "
                   "algorithmic_frac_of_peak the reference's operation count.")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
