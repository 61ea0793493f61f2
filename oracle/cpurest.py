"""ctypes front of the C++ CPU restatement (oracle/cpu_restatement.cpp, built by oracle/Makefile).

TEST INFRASTRUCTURE / CPU BASELINE ONLY: imported by tests/ and bench.py's cpu_baseline leg,
never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libcpurest.so")
_lib = None


def build(force=False):
    if force or not os.path.exists(LIB):
        subprocess.run(["make", "-C", HERE] + (["-B"] if force else []), check=True,
                       stdout=subprocess.DEVNULL)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P64, PF = C.POINTER(C.c_int64), C.POINTER(C.c_double)
        L.cpurest_run.restype = C.c_int
        L.cpurest_run.argtypes = ([C.c_int, C.c_int, C.c_int64, C.c_int64] + [P64] * 5 + [PF] * 10
                                  + [C.c_int, PF, PF])
        L.cpurest_max_threads.restype = C.c_int
        _lib = L
    return _lib


def max_threads() -> int:
    return lib().cpurest_max_threads()


def run(pk, cons, b, bi, words, state, iterations, threads=0,
        params=("0.3", "0.1", "0.7"), thresholds=(0.0, 0.0)):
    """Run `iterations` loop bodies from `state` = (x, X, y, Y) (arrays or mpf object arrays).
    Returns (completed bodies or -failure code, log (n x 8), seconds, new state)."""
    from clrsdp_amd.instance import (blocks_to_flat, concat_colmajor, flat_to_blocks, flatten,
                                     from_planes, to_planes)
    fl = flatten(cons, bi)
    ints = [np.ascontiguousarray(getattr(fl, k), dtype=np.int64)
            for k in ("m", "L", "n_samples", "delta", "ranks")]
    planes = [to_planes(concat_colmajor(fl.V), words), to_planes(np.concatenate(fl.lam), words),
              to_planes(concat_colmajor(fl.B), words), to_planes(np.concatenate(fl.c), words),
              to_planes(np.asarray(b), words)]
    x, X, y, Y = state
    st = [to_planes(np.asarray(x), words), to_planes(blocks_to_flat(X), words),
          to_planes(np.asarray(y), words), to_planes(blocks_to_flat(Y), words)]
    import mpmath
    with mpmath.workprec(320):
        pv = np.array([mpmath.mpf(str(v)) for v in params], dtype=object)
    prm = np.concatenate([to_planes(pv, words) if words > 1 else pv.astype(float),
                          np.array([float(thresholds[0]), float(thresholds[1])])])
    logs = np.zeros(8 * words * max(iterations, 1))
    secs = np.zeros(1)
    pf = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    pi = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))
    rc = lib().cpurest_run(words, threads, bi.J, bi.n_y, *[pi(a) for a in ints],
                           *[pf(a) for a in planes], *[pf(a) for a in st], pf(prm), iterations,
                           pf(logs), pf(secs))
    nx, nblk, ny = len(np.asarray(x)), len(blocks_to_flat(X)), len(np.asarray(y))
    if words == 1:
        new = (st[0], flat_to_blocks(st[1], bi), st[2], flat_to_blocks(st[3], bi))
    else:
        new = (from_planes(st[0], nx, words), flat_to_blocks(from_planes(st[1], nblk, words), bi),
               from_planes(st[2], ny, words), flat_to_blocks(from_planes(st[3], nblk, words), bi))
    n = max(rc, 0)
    if words == 1:
        log = logs[:8 * n].reshape(n, 8)
    else:   # exact limb sums (mpmath), per iteration w planes of 8 values
        log = np.array([from_planes(logs[8 * words * i:8 * words * (i + 1)], 8, words)
                        for i in range(n)], dtype=object).reshape(n, 8)
    return rc, log, float(secs[0]), new
