"""Two ranks sharing the box's GPU, clusters sharded, exchange over gloo: identical iterates to
the single-process run (up to the rank-order summation of the exchanged partials)."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("backend,J", [("gloo", 5), ("rccl", 5), ("gloo", 1)])
def test_two_ranks_match_single_rank(pk, backend, J):
    """backend "rccl": the native communicator cannot put two ranks on the box's one GPU (RCCL
    refuses with "invalid usage" on every rank), so this also covers the agreed fallback to the
    host-staged exchange; on a multi-GPU node the same worker runs the native all-gathers.
    J = 1: one rank owns no cluster (as config 5's 7 clusters on 8 GPUs) and only contributes
    neutral partials."""
    iters = 4
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "r")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CLRSDP_TEST_J=str(J))
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={_port()}",
               os.path.join(HERE, "_dist_worker.py"), out, str(iters), "iter", backend]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        res = [json.load(open(f"{out}.{k}.json")) for k in range(2)]
    cons, b = pk.synth(seed=12, J=J, delta=16, rank=1, n_y=9, m=1)
    bi = pk.get_block_info(cons)
    dev = pk.DeviceSolver(cons, b, bi)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    dev.set_state(*pk.initial_point(bi, 10.0, 10.0))
    ref = []
    for _ in range(iters):
        st = dev.iterate(P, False)
        ref.append([st.mu, st.alpha_p, st.alpha_d, st.beta_c, st.p_obj, st.d_obj])
    x, X, y, Y = dev.get_state()
    dev.close()
    for rr in res:
        np.testing.assert_allclose(np.array(rr["log"])[:, :6], np.array(ref), rtol=1e-11, atol=1e-13)
        np.testing.assert_allclose(rr["y"], y, rtol=1e-10, atol=1e-12)
    # x is sharded: each rank holds its own clusters' entries
    for rr in res:
        for j in rr["owned"]:
            a, c = bi.x_indices[j], bi.x_indices[j + 1]
            np.testing.assert_allclose(rr["x"][a:c], x[a:c], rtol=1e-10, atol=1e-12)


def test_two_ranks_full_solve_pipelined(pk):
    """solverank1sdp sharded over two ranks (pipelined host loop, device-side termination) ends
    with the single-rank synchronous run's iteration count, log and objectives."""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "s")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={_port()}",
               os.path.join(HERE, "_dist_worker.py"), out, "0", "solve"]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        res = [json.load(open(f"{out}.{k}.json")) for k in range(2)]
    cons, b = pk.synth(seed=12, J=5, delta=16, rank=1, n_y=9, m=1)
    bi = pk.get_block_info(cons)
    ref = pk.solverank1sdp(cons, b, bi, omega_p=10.0, omega_d=10.0, duality_gap_threshold=1e-6,
                           primal_error_threshold=1e-6, dual_error_threshold=1e-6,
                           verbose=False, return_info=True, pipelined=False)
    info = ref[-1]
    assert info.status == "terminated"
    for rr in res:
        assert rr["status"] == "terminated" and len(rr["log"]) == len(info.log)
        np.testing.assert_allclose(np.array(rr["log"]), np.array([r[2:] for r in info.log]),
                                   rtol=1e-9, atol=1e-12)
        assert abs(rr["d_obj"] - ref[9]) < 1e-9 and abs(rr["p_obj"] - ref[8]) < 1e-9


def test_native_rccl_one_rank_graph_equals_plain(pk):
    """The native RCCL path (clrsdp_comm_init) at world size 1: the all-gathers are issued in
    place and captured into the loop-body graph; the iterates equal a handle without a
    communicator bit for bit, through the synchronous and the pipelined loop."""
    cons, b = pk.synth(seed=5, J=4, delta=12, rank=1, n_y=7, m=1)
    bi = pk.get_block_info(cons)
    P = pk.make_params("0.3", "0.1", "0.7", 0)
    from clrsdp_amd.solver import comm_unique_id, make_control
    runs = []
    for native in (False, True):
        dev = pk.DeviceSolver(cons, b, bi)
        if native:
            dev.comm_init(comm_unique_id())
        dev.set_control(make_control("1e-15", "1e-30", "1e-30"))
        dev.set_state(*pk.initial_point(bi, 10.0, 10.0))
        dev.initial_residuals(P)
        log = []
        for _ in range(3):
            st = dev.iterate(P, False)
            log.append((st.mu, st.alpha_p, st.alpha_d, st.p_obj, st.d_obj))
        for _ in range(3):
            dev.iterate_async(P)
            st, ran = dev.iterate_wait()
            assert ran
            log.append((st.mu, st.alpha_p, st.alpha_d, st.p_obj, st.d_obj))
        x, X, y, Y = dev.get_state()
        runs.append((log, x, y))
        dev.close()
    assert runs[0][0] == runs[1][0]
    assert np.array_equal(runs[0][1], runs[1][1]) and np.array_equal(runs[0][2], runs[1][2])


def test_two_ranks_one_sided_failure_fall_back_together(pk):
    """Only rank 0's cluster has an indefinite Y, so only rank 0's S_j Cholesky fails.  The
    failure bits are OR-ed over the ranks (status_bits / status_gather with STEP's exchange), so
    both ranks skip the update, switch S_j and Q to the pivoted LU together, re-run the body and
    report the same outcome -- the reference's step-length error (cho!(Y), MPMP.jl:1846-1882),
    as the single-rank handle does on the same state."""
    from clrsdp_amd import _lib as L
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "f")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={_port()}",
               os.path.join(HERE, "_dist_worker.py"), out, "1", "failone", "gloo"]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        res = [json.load(open(f"{out}.{k}.json")) for k in range(2)]
    assert res[0]["bad"] in res[0]["owned"] and res[0]["bad"] not in res[1]["owned"]
    for rr in res:
        assert rr["code"] == L.E_STEP, rr
        assert rr["fact"] == L.FACT_FALLBACK | L.FACT_LU_SQ, rr
        assert rr["unchanged"], rr
    # the single-rank handle on the same state ends the same way
    cons, b = pk.synth(seed=12, J=5, delta=16, rank=1, n_y=9, m=1)
    bi = pk.get_block_info(cons)
    x, X, y, Y = pk.initial_point(bi, 10.0, 10.0)
    bad = res[0]["bad"]
    Y[bad] = [-0.5 * yb for yb in Y[bad]]
    dev = pk.DeviceSolver(cons, b, bi)
    try:
        dev.set_state(x, X, y, Y)
        with pytest.raises(L.ClrsdpError) as ei:
            dev.iterate(pk.make_params("0.3", "0.1", "0.7", 0), False)
        assert ei.value.code == L.E_STEP
        assert dev.factorization == L.FACT_FALLBACK | L.FACT_LU_SQ
    finally:
        dev.close()
