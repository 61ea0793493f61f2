"""World-size-2 gloo test (CPU) of the multi-GPU decomposition.

The HIP library shards clusters over ranks and all-gathers exactly these cross-cluster partials
per iteration (clrsdp.hip, `exchange` call sites): <X,Y>, Q = sum_j B_j^T S_j^-1 B_j, the
p-partials sum_j B_j^T x_j and the residual maxima, sum_j B_j^T U_j^-1 t_j (predictor and
corrector), <X+dX,Y+dY>, min lambda_min for X and Y, and <c,x>.  Here the same decomposition is
run with the oracle on each rank's clusters, the partials are all-gathered over gloo and reduced
in rank order, and the result must equal the unsharded oracle iteration.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as tmp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather(vals):
    """all_gather of a float64 vector, returned as [world, n] (the library's exchange)."""
    t = torch.tensor(np.asarray(vals, dtype=np.float64).reshape(-1))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return np.stack([o.numpy() for o in out])


def sharded_iteration(O, ar, cons_all, bi_all, owned, b, state, pd_feas, prm):
    """One loop body on this rank's clusters with the library's exchange pattern."""
    sub = [cons_all[j] for j in owned]
    bi = O.get_block_info(sub)
    x, X, y, Y = state
    dim = bi_all.total_dim
    mu = _gather([O.dot_blocks(ar, X, Y)]).sum(axis=0)[0] / dim
    mu_p = 0.0 if pd_feas else prm["beta_infeasible"] * mu
    R = O.compute_residual_R(ar, X, Y, mu_p)
    Xi = O.xinv(ar, X)
    S, AY = O.compute_S_integrated(ar, sub, Xi, Y, bi)
    lus = [ar.lu(s) for s in S]
    LinvB = [ar.solve_tril(lu, c.B[pm, :], unit=True) for (lu, pm), c in zip(lus, sub)]
    BTUinv = [ar.solve_tril(lu.T, c.B, unit=False).T for (lu, pm), c in zip(lus, sub)]
    Qp = sum(bt @ lb for bt, lb in zip(BTUinv, LinvB))
    Q = _gather(Qp).sum(axis=0).reshape(bi.n_y, bi.n_y)
    qlu, qperm = ar.lu(Q)
    dec = O.Decomposition([l for l, _ in lus], [p for _, p in lus], LinvB, BTUinv, qperm, qlu, Q, S)
    P = O.compute_weighted_A(ar, sub, x, bi)
    P = [[P[j][l] - X[j][l] for l in range(bi.L[j])] for j in range(bi.J)]
    d = O.stack_c(sub) - O.stack_B(sub) @ y - O.trace_A_AY(ar, sub, AY, bi)
    pp = sum(c.B.T @ x[bi.x_indices[j]:bi.x_indices[j + 1]] for j, c in enumerate(sub))
    p = b - _gather(pp).sum(axis=0)

    def direction(Rm):
        Z = [[O.sym(Xi[j][l] @ (P[j][l] @ Y[j][l] - Rm[j][l])) for l in range(bi.L[j])]
             for j in range(bi.J)]
        rhs = -d - O.trace_A(ar, sub, Z, bi)
        idx = bi.x_indices
        tx = [ar.solve_tril(dec.S[j], rhs[idx[j]:idx[j + 1]][dec.perms[j]], unit=True)
              for j in range(bi.J)]
        u = _gather(sum(dec.BTUinv[j] @ tx[j] for j in range(bi.J))).sum(axis=0)
        dy = ar.solve_triu(dec.Q, ar.solve_tril(dec.Q, (p - u)[dec.perm], unit=True))
        dx = np.concatenate([ar.solve_triu(dec.S[j], tx[j] + dec.LinvB[j] @ dy) for j in range(bi.J)])
        WA = O.compute_weighted_A(ar, sub, dx, bi)
        dX = [[WA[j][l] + P[j][l] for l in range(bi.L[j])] for j in range(bi.J)]
        dY = [[O.sym(Xi[j][l] @ (Rm[j][l] - dX[j][l] @ Y[j][l])) for l in range(bi.L[j])]
              for j in range(bi.J)]
        return dx, dX, dy, dY

    dx, dX, dy, dY = direction(R)
    XdX = O.block_map(lambda a, c: a + c, X, dX)
    YdY = O.block_map(lambda a, c: a + c, Y, dY)
    r = _gather([O.dot_blocks(ar, XdX, YdY)]).sum(axis=0)[0] / (mu * dim)
    beta = r * r if r < 1 else r
    beta_c = max(prm["beta_infeasible"], beta) if not pd_feas else min(max(prm["beta_feasible"], beta), 1.0)
    R2 = O.compute_residual_R(ar, X, Y, beta_c * mu, dX, dY)
    dx, dX, dy, dY = direction(R2)

    def mineig(M, dM):
        e = []
        for j in range(bi.J):
            for l in range(bi.L[j]):
                Lc = ar.cholesky(M[j][l])
                T = ar.solve_tril(Lc, dM[j][l], unit=False)
                T = ar.solve_tril(Lc, T.T.copy(), unit=False)
                e.append(min(ar.eigvals_real(T)))
        return min(e)

    mins = _gather([mineig(X, dX), mineig(Y, dY)]).min(axis=0)
    g = prm["gamma"]
    ap = 1.0 if mins[0] > -g else -g / mins[0]
    ad = 1.0 if mins[1] > -g else -g / mins[1]
    if pd_feas:
        ap = ad = min(ap, ad)
    x = x + ap * dx
    y = y + ad * dy
    X = O.block_map(lambda a, c: a + ap * c, X, dX)
    Y = O.block_map(lambda a, c: a + ad * c, Y, dY)
    pobj = _gather([O.dot_c(ar, sub, x)]).sum(axis=0)[0]
    return (x, X, y, Y), dict(mu=mu, alpha_p=ap, alpha_d=ad, beta_c=beta_c, p_obj=pobj)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import _clrsdp_pkg
        from oracle import mpmp_oracle as O
        pk = _clrsdp_pkg.load()
        cons, b = pk.synth(seed=11, J=5, delta=4, rank=1, n_y=3, m=2, L=1)
        bi_all = O.get_block_info(cons)
        owned = pk.partition_clusters(pk.get_block_info(cons), world)[rank]
        ar = O.Fp64()
        prm = {k: O._param(ar, v) for k, v in O.DEFAULTS.items()}
        sub = [cons[j] for j in owned]
        bi = O.get_block_info(sub)
        st = O.initial_point(ar, bi, 10.0, 10.0)
        logs = []
        for _ in range(3):
            st, inter = sharded_iteration(O, ar, cons, bi_all, owned, b, st, False, prm)
            logs.append([inter[k] for k in ("mu", "alpha_p", "alpha_d", "beta_c", "p_obj")])
        q.put((rank, owned, logs, [np.asarray(v) for v in st[0:1]], st[2]))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_iteration_matches_single(pk, oracle):
    world = 2
    port = _free_port()
    ctx = tmp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get() for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    # single-process reference
    cons, b = pk.synth(seed=11, J=5, delta=4, rank=1, n_y=3, m=2, L=1)
    bi = oracle.get_block_info(cons)
    ar = oracle.Fp64()
    prm = {k: oracle._param(ar, v) for k, v in oracle.DEFAULTS.items()}
    st = oracle.initial_point(ar, bi, 10.0, 10.0)
    ref = []
    for _ in range(3):
        st, it = oracle.iteration(ar, cons, bi, b, None, 0.0, st, False, prm)
        ref.append([it["mu"], it["alpha_p"], it["alpha_d"], it["beta_c"],
                    oracle.primal_objective(ar, cons, st[0], 0.0)])
    for r in range(world):
        np.testing.assert_allclose(np.array(res[r][2]), np.array(ref), rtol=1e-11)
        np.testing.assert_allclose(res[r][4], st[2], rtol=1e-10, atol=1e-12)
    # x is sharded: reassemble by cluster ownership
    x = np.zeros(sum(bi.dim_S))
    for r in range(world):
        owned = res[r][1]
        off = 0
        for j in owned:
            D = bi.dim_S[j]
            x[bi.x_indices[j]:bi.x_indices[j] + D] = res[r][3][0][off:off + D]
            off += D
    np.testing.assert_allclose(x, st[0], rtol=1e-10, atol=1e-12)
