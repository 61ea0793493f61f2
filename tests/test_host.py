"""CPU tests of the host side: the C-ABI library loads and exports every symbol of
include/clrsdp.h (no compute call without a GPU), limb splitting, layouts, the balancer."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol(pk):
    hdr = open(os.path.join(ROOT, "include", "clrsdp.h")).read()
    declared = sorted(set(re.findall(r"\b(clrsdp_[a-z_]+)\s*\(", hdr)))
    assert "clrsdp_iterate" in declared and len(declared) >= 15
    lib = pk._lib.lib()
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(pk._lib.EXPORTS) == declared
    assert lib.clrsdp_version() >= 100


def test_library_rejects_bad_arguments_without_gpu(pk):
    """Argument validation happens before any HIP call, so it can run here."""
    L = pk._lib
    lib = L.lib()
    h = ctypes.c_void_p()
    assert lib.clrsdp_create(None, None, ctypes.byref(h)) == L.E_ARG
    assert lib.clrsdp_iterate(None, None, 0, None) == L.E_ARG
    assert b"null" in lib.clrsdp_last_error(None)
    assert lib.clrsdp_destroy(None) == L.OK


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "clustered-low-rank-sdp-solver_amd")
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            src = open(os.path.join(pkg, fn)).read()
            assert "oracle" not in re.sub(r'""".*?"""', "", src, flags=re.S).replace("# ", ""), fn


def test_planar_limbs_are_exact(pk):
    import mpmath
    from clrsdp_amd.instance import to_planes
    mpmath.mp.prec = 256
    vals = np.array([mpmath.mpf(1) / 3, -mpmath.pi, mpmath.mpf("1e-40"), mpmath.mpf(0)],
                    dtype=object)
    for w in (1, 2, 4):
        P = to_planes(vals, w).reshape(w, -1)
        for i, v in enumerate(vals):
            s = mpmath.mpf(0)
            for q in range(w):
                s += mpmath.mpf(P[q, i])
            assert abs(s - v) <= abs(v) * mpmath.mpf(2) ** (-52 * w) + mpmath.mpf(1e-300)
        if w > 1:  # limbs are non-overlapping: |lo| <= ulp(hi)/2
            assert np.all(np.abs(P[1]) <= np.abs(P[0]) * 2.0 ** -52 + 1e-300)


def test_flat_layout_matches_reference_hcat(pk):
    """V of block (j,l) is the hcat of v_{j,l,k,rnk} in (k, rnk) order (MPMP.jl:1249-1254)."""
    from clrsdp_amd.instance import flatten, concat_colmajor
    cons, b = pk.synth(seed=2, J=2, delta=3, rank=1, n_y=2, m=2, L=2,
                       ranks=[[1, 2, 0, 1, 1], [1, 1, 1, 1, 3]], N=5)
    bi = pk.get_block_info(cons)
    fl = flatten(cons, bi)
    assert list(fl.ranks[:5]) == [1, 2, 0, 1, 1]
    assert fl.V[0].shape == (3, 5) and fl.V[1].shape == (3, 7)
    np.testing.assert_array_equal(fl.V[0][:, 2], cons[0].A[0][1][1])
    assert fl.block_sizes == [6, 6, 6, 6]
    allv = concat_colmajor(fl.V)
    assert allv.size == sum(v.size for v in fl.V)


def test_partition_clusters_balanced_and_complete(pk):
    for cfg, world in [(dict(J=64, delta=8, rank=1, n_y=4), 8), (dict(J=7, delta=4, rank=1, n_y=2), 8),
                       (dict(J=5, delta=4, rank=1, n_y=2), 2)]:
        cons, b = pk.synth(seed=0, **cfg)
        bi = pk.get_block_info(cons)
        parts = pk.partition_clusters(bi, world)
        assert len(parts) == world
        assert sorted(c for p in parts for c in p) == list(range(bi.J))
        if cfg["J"] % world == 0:
            assert all(len(p) == cfg["J"] // world for p in parts)


def test_bench_algorithmic_counts():
    import bench
    import _clrsdp_pkg
    pk = _clrsdp_pkg.load()
    cons, b = pk.synth(seed=0, J=2, delta=8, rank=1, n_y=4)
    bi = pk.get_block_info(cons)
    fl, by = bench.schur_flops_bytes(bi)
    d, K, D = 8, 15, 15
    assert fl == 2 * (4.0 * d * K * (d + K) + 8.0 * D * (D + 1) / 2)
    assert by == 2 * 8 * (2 * d * d + d * K + K + D * (D + 1) / 2 + K)


MW_PROBE = r"""
#include "mwfloat.h"
#include <cstdio>
#include <cstdlib>
using namespace mw;
template <class T> T rnd(unsigned& s) {
  T v = T(0.0); double sc = 1.0;
  for (int q = 0; q < Num<T>::W; ++q) {
    s = s * 1664525u + 1013904223u;
    v += T(((double)(s >> 8) / 16777216.0 - 0.5) * sc); sc *= 1e-16;
  }
  return v;
}
template <class T> void pr(const T& v) {
  const double* d = reinterpret_cast<const double*>(&v);
  for (int q = 0; q < Num<T>::W; ++q) printf(" %a", d[q]);
}
template <class T> void run(unsigned s) {
  for (int t = 0; t < 40; ++t) {
    T a = rnd<T>(s), b = rnd<T>(s);
    T acc = a; for (int k = 0; k < 5; ++k) acc += b;   // loop-carried sums
    T r[7] = {a + b, a - b, a * b, a / b, Num<T>::sqrt_(a * a), a * T(-3.0), acc};
    pr(a); pr(b); for (auto& v : r) pr(v); printf("\n");
  }
}
int main() { run<dd>(7u); run<qd>(11u); }
"""


def test_multiword_arithmetic_against_mpmath(tmp_path):
    """dd / qd arithmetic of mwfloat.h (host build of the device code) against 320-bit mpmath:
    add/sub/mul/div/sqrt within a few units of 2^-104 (dd) and 2^-208 (qd)."""
    import shutil
    import subprocess
    import mpmath
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    src = tmp_path / "mw.cpp"
    src.write_text(MW_PROBE)
    exe = tmp_path / "mw"
    inc = os.path.join(ROOT, "clustered-low-rank-sdp-solver_amd", "csrc")
    subprocess.run([cxx, "-x", "c++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", "-I" + inc, str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    mpmath.mp.prec = 320
    for words, lines, tol in ((2, out[:40], 2.0 ** -100), (4, out[40:80], 2.0 ** -203)):
        for ln in lines:
            v = [mpmath.mpf(float.fromhex(t)) for t in ln.split()]
            vals = [sum(v[i:i + words]) for i in range(0, len(v), words)]
            a, b = vals[0], vals[1]
            exp = [a + b, a - b, a * b, a / b, abs(a), a * -3, a + 5 * b]
            for got, e in zip(vals[2:], exp):
                assert abs(got - e) <= tol * max(abs(e), abs(a), abs(b)), (words, float(got), float(e))


def test_planar_limbs_exact_at_default_mpmath_precision(pk):
    """to_planes/from_planes must not depend on the global mpmath precision (prepareabc output
    carries its own 512-bit values; a 53-bit remainder would silently drop limbs 3 and 4)."""
    import mpmath
    from clrsdp_amd.instance import from_planes, to_planes
    old = mpmath.mp.prec
    try:
        with mpmath.workprec(512):
            v = np.array([mpmath.sqrt(2) / 3, -mpmath.mpf(1) / 7, mpmath.exp(40)], dtype=object)
        mpmath.mp.prec = 53
        back = from_planes(to_planes(v, 4), 3, 4)
        with mpmath.workprec(512):
            err = max(abs(a - b) / abs(a) for a, b in zip(v, back))
        assert err < mpmath.mpf(2) ** -205
        assert float(to_planes(np.array([mpmath.pi], dtype=object), 4)[3]) != 0.0
    finally:
        mpmath.mp.prec = old


def test_time_spent_report_groups_stages_like_the_reference(pk):
    """solverank1sdp's closing report (MPMP.jl:973-1012): the device stages are summed into the
    reference's groups (Decomp = Schur + factorisation, R = both R computations, ...)."""
    from clrsdp_amd import _lib
    from clrsdp_amd.solver import _stage_groups, _time_spent
    ph = np.arange(1, _lib.NUM_STAGES + 1, dtype=float)
    g = _stage_groups(ph)
    S = dict(zip(_lib.STAGE_NAMES, ph))
    assert g["Decomp"] == S["schur"] + S["factor"] and g["R"] == S["mu_R"] + S["corrector_R"]
    assert g["alpha"] == S["step"] and g["predict_dir"] == S["predictor"]
    assert sum(g.values()) == ph.sum()
    txt = _time_spent(2.0, ph)
    assert "Time spent" in txt and "Decomp" in txt and "Time inside decomp" in txt
    assert "timing=True" in _time_spent(2.0, None)


def test_time_spent_report_prints_the_reference_inner_buckets(pk):
    """With the inner buckets (clrsdp_iter_stats.inner_ms) the report has MPMP.jl:997-1012's two
    inner tables: schur / chol_S / comp CinvB / comp Q / chol_Q and calc Z ... calc dY."""
    from clrsdp_amd import _lib
    from clrsdp_amd.solver import _time_spent
    assert _lib.NUM_INNER == len(_lib.INNER_NAMES) == 10
    ph = np.ones(_lib.NUM_STAGES)
    txt = _time_spent(1.0, ph, np.arange(1.0, 11.0))
    for h in ("chol_S", "comp CinvB", "comp Q", "chol_Q", "calc Z", "calc rhs x", "solve system",
              "calc dX", "calc dY", "Time inside search directions"):
        assert h in txt
    assert "1.00000e+01" in txt   # the last bucket (calc dY)


def test_iter_stats_layout_matches_the_header(pk):
    """The ctypes mirror of clrsdp_iter_stats has the header's fields in order (the full-width
    loop-control limbs and the inner buckets were appended in round 4)."""
    import re
    from clrsdp_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "clrsdp.h")).read()
    body = re.search(r"typedef struct \{([^}]*)\} clrsdp_iter_stats;", hdr, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"(\w+)(?:\[[^\]]*\])?;", body)
    assert names == [f[0] for f in _lib.IterStats._fields_]


def test_device_thresholds_are_exact_limb_sums():
    """Loop control at dd/qd compares against the threshold the device holds (the first w limbs
    of the decimal string, summed exactly), so 1e-20 is not rounded to fp64 on the host."""
    import mpmath
    from clrsdp_amd.solver import device_threshold, limbs
    assert device_threshold("1e-24", 1) == float("1e-24")
    for w in (2, 4):
        t = device_threshold("1e-24", w)
        assert isinstance(t, mpmath.mpf)
        with mpmath.workprec(400):
            assert t == mpmath.fsum(limbs("1e-24")[:w])
            assert abs(t - mpmath.mpf("1e-24")) < mpmath.mpf("1e-24") * mpmath.mpf(2) ** (-52 * w)
    # a gap a few ulps of fp64 below the threshold is decided correctly at dd
    g = device_threshold("1e-24", 2) * (1 - mpmath.mpf(2) ** -80)
    assert g < device_threshold("1e-24", 2) and not float(g) < float("1e-24") * (1 - 2 ** -52)


def test_return_and_log_types_per_precision(pk):
    """The public types of solverank1sdp's outputs: the iteration log holds plain
    floats except the gap column, which keeps the loop control's type (a float at fp64, the
    full-width mpmath number at dd/qd that device_threshold's exact comparisons use), and the
    docstring states that the returned gap and objectives are mpmath numbers at dd/qd and floats
    at fp64."""
    import types

    import mpmath
    from clrsdp_amd import solver
    st = types.SimpleNamespace(mu=0.5, P_err=1e-3, p_err=2e-3, d_err=3e-3, alpha_p=0.7,
                               alpha_d=0.8, beta_c=0.1)
    for gap in (1e-5, np.float64(2e-7), mpmath.mpf("1e-25"), solver.device_threshold("1e-20", 2)):
        row = solver.log_row(3, 0.25, st, mpmath.mpf("1.5"), 1.25, gap)
        assert type(row[0]) is int and all(type(v) is float for i, v in enumerate(row) if i not in (0, 5))
        assert row[5] == gap
        assert type(row[5]) is (mpmath.mpf if isinstance(gap, mpmath.mpf) else float)
    doc = solver.solverank1sdp.__doc__
    assert "mpmath numbers" in doc and "at fp64 they are floats" in doc


def test_keyword_generators(pk):
    """synth_C is exactly symmetric in X's block structure; synth_start is strictly positive
    definite (diagonally dominant) and deterministic."""
    cons, b = pk.synth(J=2, delta=3, rank=1, n_y=3, m=2, L=2, seed=4)
    bi = pk.get_block_info(cons)
    C = pk.synth_C(bi, 21)
    assert [[c.shape[0] for c in row] for row in C] == bi.Y_blocksizes
    assert all(np.array_equal(c, c.T) and np.any(c != 0) for row in C for c in row)
    x, X, y, Y = pk.synth_start(bi, 5)
    x2, X2, y2, Y2 = pk.synth_start(bi, 5)
    assert np.array_equal(x, x2) and np.array_equal(Y[1][0], Y2[1][0])
    assert len(x) == sum(bi.dim_S) and len(y) == bi.n_y
    for M in [m for row in X + Y for m in row]:
        assert np.array_equal(M, M.T) and np.linalg.eigvalsh(M).min() > 0.5


def test_round4_goldens_are_consistent():
    """The keyword goldens carry their keywords and stop as their thresholds say; the gap-1e-20
    golden terminates with the final gap below 1e-20 and the previous one above it (so the
    double-double loops have an unambiguous iteration to stop at)."""
    import json
    import mpmath
    gd = os.path.join(ROOT, "tests", "golden")
    with mpmath.workprec(256):
        g = json.load(open(os.path.join(gd, "rank2_mp256_seed5_gap20.json")))
        assert g["status"] == "terminated"
        thr = mpmath.mpf(g["params"]["duality_gap_threshold"])
        assert mpmath.mpf(g["final"]["gap"]) < thr < mpmath.mpf(g["log"][-1]["gap"])
        assert all(mpmath.mpf(r["gap"]) > thr for r in g["log"][1:])
        for name, kw in (("kw_C_b0_mp256", "C_seed"), ("kw_needp_mp256", "need_primal_feasible"),
                         ("kw_needd_mp256", "need_dual_feasible"), ("kw_start_mp256", "start_seed")):
            k = json.load(open(os.path.join(gd, name + ".json")))
            assert kw in k["keywords"]
        p = json.load(open(os.path.join(gd, "kw_needp_mp256.json")))
        assert p["status"] == "terminated" and len(p["log"]) < p["iterations"]
        last = p["log"][-1]
        assert max(mpmath.mpf(last["P_err"]), mpmath.mpf(last["p_err"])) < \
            mpmath.mpf(p["params"]["primal_error_threshold"])
