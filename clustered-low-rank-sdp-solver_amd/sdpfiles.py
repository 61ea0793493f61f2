"""On-disk instance format: ``write_files`` / ``read_files``.

SpherePacking.jl calls ``write_files(file_path, constraints, blockinfo, b)`` from the package
WriteFilesSDPB (SP.jl:6, 95-98), which is not part of the reference (not vendored, no version
pinned).  Its exact schema is therefore unknown; this module writes the same information in
an SDPB-style directory of JSON files, one set per cluster.  Multi-precision numbers are
written exactly as "<mantissa>p<exponent>" (binary mantissa and exponent as integers), floats
by their shortest round-trip repr, so a ``read_files`` round trip is bit-exact at any
precision:

    <dir>/control.json          {"num_clusters", "n_y", "format", "precision_bits"}
    <dir>/objectives.json       {"b": [...], "b0": "0"}
    <dir>/block_info_<j>.json   {"m", "L", "num_points", "delta": [...], "ranks": [[...]]}
    <dir>/free_var_matrix_<j>.json  {"rows": D, "cols": n_y, "elements": [[row]...]}  (B_j)
    <dir>/primal_objective_c_<j>.json  {"c": [...]}
    <dir>/bilinear_bases_<j>.json {"vectors": [l][k][r] -> [...], "eigenvalues": [l][k][r]}

The constraint tuple is the ``(A, B, c, H)`` of ``prepareabc`` (MPMP.jl:385-406).
"""
from __future__ import annotations

import json
import os
from typing import List, Tuple

import mpmath
import numpy as np

from .blockinfo import BlockInfo, get_block_info
from .instance import Cluster

FORMAT = "clrsdp-sdpb-style-1"


def _s(v) -> str:
    if isinstance(v, (float, np.floating)):
        return repr(float(v))
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if not isinstance(v, mpmath.mpf):
        with mpmath.workprec(1024):
            v = mpmath.mpf(v)
    return _exact(v)


def _exact(v) -> str:
    """Exact encoding of a binary mpf as "<mantissa>p<exponent>" (value = mantissa * 2^exponent)."""
    if v == 0:
        return "0p0"
    sign, man, exp, _ = v._mpf_
    return f"{'-' if sign else ''}{int(man)}p{int(exp)}"


def _parse(s: str, exact: bool):
    if "p" in s:
        man, exp = (int(t) for t in s.split("p"))
        with mpmath.workprec(max(53, abs(man).bit_length())):   # exact, whatever mp.prec is
            v = mpmath.mpf((man, exp)) if man != 0 else mpmath.mpf(0)
        return v if exact else float(v)
    return mpmath.mpf(s) if exact else float(s)


def _prec_of(constraints) -> int:
    """Largest significand width (bits) among the c entries (53 for float data)."""
    bits = 53
    for cl in constraints:
        for v in np.asarray(cl.c).reshape(-1):
            if isinstance(v, mpmath.mpf) and v != 0:
                bits = max(bits, int(v._mpf_[3]))
    return bits


def write_files(file_path: str, constraints, blockinfo: BlockInfo, b, b0=0) -> None:
    """Write the instance (constraints, b) under directory ``file_path`` (SP.jl:95-98)."""
    os.makedirs(file_path, exist_ok=True)
    bi = blockinfo
    obj = lambda name, d: json.dump(d, open(os.path.join(file_path, name), "w"))
    obj("control.json", {"num_clusters": bi.J, "n_y": bi.n_y, "format": FORMAT,
                         "precision_bits": _prec_of(constraints)})
    obj("objectives.json", {"b": [_s(v) for v in np.asarray(b).reshape(-1)], "b0": _s(b0)})
    for j, cl in enumerate(constraints):
        B = np.asarray(cl.B)
        obj(f"block_info_{j}.json", {
            "m": bi.m[j], "L": bi.L[j], "num_points": bi.n_samples[j],
            "delta": [bi.Y_blocksizes[j][l] // bi.m[j] for l in range(bi.L[j])],
            "ranks": bi.ranks[j]})
        obj(f"free_var_matrix_{j}.json", {"rows": int(B.shape[0]), "cols": int(B.shape[1]),
                                          "elements": [[_s(v) for v in row] for row in B]})
        obj(f"primal_objective_c_{j}.json", {"c": [_s(v) for v in np.asarray(cl.c).reshape(-1)]})
        obj(f"bilinear_bases_{j}.json", {
            "vectors": [[[[_s(x) for x in np.asarray(v).reshape(-1)] for v in Ak] for Ak in Al]
                        for Al in cl.A],
            "eigenvalues": [[[_s(h) for h in Hk] for Hk in Hl] for Hl in cl.H]})


def read_files(file_path: str, exact: bool = True) -> Tuple[List[Cluster], np.ndarray, BlockInfo]:
    """Read an instance written by :func:`write_files`.  ``exact``: mpmath values (object
    arrays) as written; otherwise float64.  Returns ``(constraints, b, blockinfo)``."""
    load = lambda name: json.load(open(os.path.join(file_path, name)))
    ctl = load("control.json")
    if ctl.get("format") != FORMAT:
        raise ValueError(f"{file_path}: unknown format {ctl.get('format')!r}")
    conv = (lambda s: _parse(s, exact))
    dt = object if exact else np.float64
    ob = load("objectives.json")
    b = np.array([conv(s) for s in ob["b"]], dtype=dt)
    cons = []
    for j in range(ctl["num_clusters"]):
        fv = load(f"free_var_matrix_{j}.json")
        B = np.empty((fv["rows"], fv["cols"]), dtype=dt)
        for r, row in enumerate(fv["elements"]):
            B[r, :] = [conv(s) for s in row]
        c = np.array([conv(s) for s in load(f"primal_objective_c_{j}.json")["c"]], dtype=dt)
        bb = load(f"bilinear_bases_{j}.json")
        A = [[[np.array([conv(s) for s in v], dtype=dt) for v in Ak] for Ak in Al]
             for Al in bb["vectors"]]
        H = [[[conv(s) for s in Hk] for Hk in Hl] for Hl in bb["eigenvalues"]]
        cons.append(Cluster(A, B, c, H))
    bi = get_block_info(cons)
    if bi.n_y != ctl["n_y"]:
        raise ValueError(f"{file_path}: n_y mismatch ({bi.n_y} vs {ctl['n_y']})")
    return cons, b, bi
