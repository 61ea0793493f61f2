"""Benchmark: interior-point iterations/s of solverank1sdp's loop body on MI355X.

Workload (BASELINE.json configs[2], the north-star instance): synthetic clustered low-rank SDP,
64 clusters x 128x128 blocks (m = 1, L = 1, delta = 128), rank-1 constraints, N = 255 samples per
cluster, n_y = 128, fp64 -- SURVEY.md §8d "C3".  One step = one full predictor-corrector
iteration (MPMP.jl:755-887) on device-resident data.

With --gpus N (one process per GPU, clusters balanced as MPMP.jl:425-465, the cross-cluster
partials all-gathered over RCCL) the default is the configuration as BASELINE.json states it:
the 64-cluster instance sharded over the N GPUs (STRONG scaling, 8 clusters per GPU at N = 8);
`value` is the instance's iterations/s, the whole job's throughput.  --scaling weak gives every
GPU a C3-sized shard (J = 64 N clusters coupled by n_y = 128); `value` is then that instance's
iterations/s and `shard_iterations_per_s_summed` = N x value.

Also reported: the Schur-assembly roofline (its kernels timed on the device clock inside the
timed region), and a CPU baseline: the C++/OpenMP restatement of the reference algorithm
(oracle/cpu_restatement.cpp) at the bench's word type on the host's cores, rank 0 at N = 1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (J, delta, rank, n_y, m, L)
    "c3": dict(J=64, delta=128, rank=1, n_y=128),
    "c2": dict(J=16, delta=64, rank=2, n_y=64),
    "c1": dict(J=2, delta=4, rank=1, n_y=4),
    # config 5 shape (sphere packing): 7 clusters, blocks {2}, {18,16}, {9,8}x3,
    # {1}x2, dim_S {3,51,17,17,17,1,1}, n_y = 52 -- run with --precision 4 (quad-double)
    "c5": dict(kind="sphere_packing_shape"),
}
DTYPES = {1: "f64", 2: "dd(f64x2)", 4: "qd(f64x4)"}
FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X fp64 matrix spec; measured ceiling 72.4 (profiles/r01_f64_mfma_probe.log)
HBM_PEAK_GBS = 8000.0
# multi-word runs (dd, qd) compute on the fp64 VALU: measured multiply-add ceilings x 2 flops
# (tools/micro/mw_peak.hip -> profiles/r01_mw_peak.log: dd 1.868 T/s, qd 0.349 T/s; fp64 FMA
# 30.2 T/s, so a dd multiply-add costs 16.2 and a qd one 86.5 fp64 FMA slots)
MW_VALU_PEAK_TFLOPS = {2: 3.736, 4: 0.698}
# double-double Schur products of m = 1 blocks on the int8 matrix cores (Ozaki scheme, round 6,
# oz_gemm in kernels_dense.h): every double-double multiply-add of the product costs 136 int8
# multiply-adds (16 digits per operand, the 136 digit pairs of levels 0..15).  Dense int8 MFMA
# peak 5.0 POPS (2x the ~2.5 PF dense BF16 rate per clock, /opt/skills/guides/MI355X_MICROARCH.md
# "Matrix cores"), so the stage's ceiling in double-double flops is 2 x 5.0e15 / 2 / 136.
I8_MFMA_PEAK_TOPS = 5000.0
OZAKI_DIGIT_PAIRS = 136
OZAKI_DD_PEAK_TFLOPS = 2 * (I8_MFMA_PEAK_TOPS / 2) / OZAKI_DIGIT_PAIRS


def env_on(name):
    """The library's switch rule (clrsdp.hip env_on): set, and not starting with '0'."""
    v = os.environ.get(name)
    return v is not None and v[:1] != "0"


def schur_flops_bytes(bi, word=8):
    """Algorithmic Schur-assembly work of one iteration: per (j,l) block
    4 m^2 delta K (delta + K) + 8 rank^2 D(D+1)/2 flops and
    word * [2 n^2 + delta K + K + D(D+1)/2 + m(m+1)/2 K] bytes."""
    fl, by = 0.0, 0.0
    for j in range(bi.J):
        m, D = bi.m[j], bi.dim_S[j]
        for l in range(bi.L[j]):
            n = bi.Y_blocksizes[j][l]
            d = n // m
            K = bi.rank_sums[j][l][-1]
            rk = max(bi.ranks[j][l])
            fl += 4.0 * m * m * d * K * (d + K) + 8.0 * rk * rk * D * (D + 1) / 2
            by += word * (2 * n * n + d * K + K + D * (D + 1) / 2 + m * (m + 1) / 2 * K)
    return fl, by


def schur_pmc_traffic(config, precision, world, clusters=0):
    """HBM bytes per iteration of the Schur stage (FETCH_SIZE + WRITE_SIZE of its launches) from
    the newest committed PMC summary, profiles/rNN_schur_pmc.json (tools/profile_round.sh, the
    default C3 fp64 1-GPU run), used only when it was taken on this very build (its
    source_hash); otherwise None and the source says why.  None for other runs."""
    import glob
    if config != "c3" or precision != 1 or world != 1 or clusters not in (0, 64):
        return None, None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_schur_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    import _clrsdp_pkg
    cur = _clrsdp_pkg.load_build().source_hash()
    src = os.path.relpath(files[-1], ROOT)
    if d.get("source_hash") != cur:
        return None, (f"stale: {src} was counted on build {d.get('source_hash')}, this is build "
                      f"{cur} (run tools/profile_round.sh)")
    return d.get("traffic_bytes_per_iteration"), f"{src} (build {cur})"


def schur_pmc_issued(config, precision, world, clusters=0):
    """The fp64 MFMA work the Schur kernel actually issues, as a fraction of peak
    (SQ_INSTS_VALU_MFMA_F64 x 2048 flop over its average duration, tools/pmc_kernels.py), from the
    newest committed profiles/rNN_kernels_pmc.json taken on this very build, beside `frac`, which
    prices the launch on the reference's redundant algorithmic flop count.  The
    fused kernel skips the lower tiles and the symmetric half of the pairing, so it issues fewer
    flops than that count.  None (with the reason) otherwise."""
    import glob
    if config != "c3" or precision != 1 or world != 1 or clusters not in (0, 64):
        return None, None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_kernels_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    import _clrsdp_pkg
    cur = _clrsdp_pkg.load_build().source_hash()
    src = os.path.relpath(files[-1], ROOT)
    if d.get("source_hash") != cur:
        return None, f"stale: {src} was counted on build {d.get('source_hash')}, this is build {cur}"
    k = d.get("kernels", {}).get("schur_fused_f64")
    if not k:
        return None, f"{src} holds no schur_fused_f64 record"
    return k.get("issued_frac_of_peak"), f"{src} (build {cur}): schur_fused_f64 MFMA instructions issued"


def cpu_baseline(pk, cons, b, bi, precision=1, budget_s=15.0):
    """Time the C++/OpenMP restatement of the reference algorithm (oracle/cpu_restatement.cpp:
    the same loop body as MPMP.jl:755-887 with approx_lu! for S_j and Q, threaded over the
    reference's (j,l) and cluster partitions) on this instance at the bench's word type
    (double, double-double, quad-double), on all the host threads OpenMP is given
    (OMP_NUM_THREADS), from the reference's initial point: one calibration body, then as many
    as fit in ~budget_s."""
    from oracle import cpurest
    cpurest.build()
    threads = cpurest.max_threads()
    st = pk.initial_point(bi, 100.0, 100.0)
    rc, _, s1, st1 = cpurest.run(pk, cons, b, bi, precision, st, 1)
    if rc != 1:
        return {"value": None, "unit": "iterations/s", "cores": threads, "kind": "port",
                "sample": f"the C++ restatement failed in its first loop body (code {rc})"}
    n = int(max(1, min(30, budget_s / max(s1, 1e-3))))
    rc, _, secs, _ = cpurest.run(pk, cons, b, bi, precision, st1, n)
    n = max(rc, 0)
    return {"value": n / secs if n else None, "unit": "iterations/s", "cores": threads,
            "kind": "port",
            "sample": (f"{n} loop bodies (iterations 2..{n + 1}) of the same instance from the "
                       f"reference's initial point; C++/OpenMP restatement of MPMP.jl's loop body "
                       f"(oracle/cpu_restatement.cpp) at {DTYPES[precision]}, {threads} OpenMP threads")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--precision", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--loop", choices=["auto", "sync", "pipelined"], default="auto",
                    help="host loop: wait for every loop body (sync; hipGraph replay, faster at one "
                         "GPU: 1.13-1.15 vs 1.15-1.17 ms measured) or stay one body behind "
                         "(pipelined; auto = pipelined when the clusters are sharded)")
    ap.add_argument("--clusters", type=int, default=0,
                    help="override J of the config (per-rank sizing experiments; not a bench line)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="N > 1: strong = the config's J sharded over the GPUs (BASELINE.json "
                         "configs[2], the default), weak = one config-sized shard per GPU (J x N "
                         "clusters)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("CLRSDP_BENCH_ONE_GPU"):
        # rehearsal of the multi-rank bench on a one-GPU box: every rank on device 0 (RCCL then
        # refuses the communicator and the exchange falls back to host-staged gloo, loudly)
        local_rank = 0
    import _clrsdp_pkg
    pk = _clrsdp_pkg.load()
    from clrsdp_amd import _lib

    cfg = dict(CONFIGS[args.config])
    if args.clusters:
        cfg["J"] = args.clusters
    weak = world > 1 and args.scaling == "weak" and "J" in cfg
    if weak:
        cfg["J"] *= world   # one config-sized shard of clusters per GPU
    if cfg.get("kind") == "sphere_packing_shape":
        cons, b = pk.synth_mixed(**pk.SPHERE_PACKING_SHAPE, seed=args.seed)
    else:
        cons, b = pk.synth(seed=args.seed, **cfg)
    bi = pk.get_block_info(cons)
    parts = pk.partition_clusters(bi, world)
    owned = parts[rank] if world > 1 else None

    dist = None
    if world > 1:
        from clrsdp_amd import dist as cdist
        dist = cdist.make_exchange(local_rank)
    dev = pk.DeviceSolver(cons, b, bi, precision_words=args.precision, device=local_rank,
                          rank=rank, world=world, owned=owned, timing=False)
    if dist is not None:
        dist.attach(dev)
    prm = pk.make_params("0.3", "0.1", "0.7", 0)
    from clrsdp_amd.solver import make_control
    # the reference's default thresholds (MPMP.jl:607-609); loop control on the device
    dev.set_control(make_control("1e-15", "1e-30", "1e-30"))
    x0, X0, y0, Y0 = pk.initial_point(bi, 100.0, 100.0)
    dev.set_state(x0, X0, y0, Y0)
    dev.initial_residuals(prm)

    # check_pd_feasibility (MPMP.jl:949-953) with the thresholds set above, from the previous
    # body's log row, as solverank1sdp's synchronous loop does
    PTHR = DTHR = 1e-30
    feas = [False]

    last_mu = [1.0]

    def step():   # one synchronous loop body
        st = dev.iterate(prm, feas[0])
        feas[0] = max(st.p_err, st.P_err) < PTHR and st.d_err < DTHR
        last_mu[0] = st.mu
        return st

    pipelined = args.loop == "pipelined" or (args.loop == "auto" and world > 1)

    # Every RESTART bodies the iterate goes back to the snapshot taken after the warm-up (a
    # device-side copy, stream-ordered): the instance stagnates near mu ~ 1e-12 after ~100
    # iterations and the fp64 factorisations break down after ~250, so a long --steps window
    # replays iterations 1..RESTART instead.  Every timed step is still one full loop body.
    # Also back to the snapshot once mu falls below MU_FLOOR (the last body's mu read back; in
    # the pipelined loop the body before it): the smaller shards (--clusters 8) reach the stagnation regime (mu ~ 4e-12, dual steps
    # ~1e-3) by iteration ~60, where a loss of definiteness of Y depends on the rounding of
    # single operations -- a healthy window for every shard size.
    RESTART = 64
    MU_FLOOR = 1e-8
    count = [0]
    # restarts per cause (period / mu floor), reported in the JSON for the timed window
    restarts = {"period": 0, "mu_floor": 0}

    def maybe_restart():
        count[0] += 1
        if count[0] % RESTART == 0 or last_mu[0] < MU_FLOOR:
            restarts["period" if count[0] % RESTART == 0 else "mu_floor"] += 1
            dev.restore_state()
            feas[0] = False   # the snapshot is the (infeasible) initial point
            last_mu[0] = 1.0

    def run_bodies(n):
        """n loop bodies as solverank1sdp runs them: the host one body behind the device
        (clrsdp_iterate_async / _wait), every log row read back."""
        if not pipelined:
            for _ in range(n):
                step()
                maybe_restart()
            return
        inflight = 0
        for _ in range(n):
            dev.iterate_async(prm)
            maybe_restart()
            inflight += 1
            if inflight == 2:
                st, ran = dev.iterate_wait()
                inflight -= 1
                if not ran:
                    raise RuntimeError("solver terminated inside the benchmark window")
                last_mu[0] = st.mu   # (one body behind: the MU_FLOOR restart comes a body later)
        while inflight:
            _, ran = dev.iterate_wait()
            inflight -= 1
            if not ran:
                raise RuntimeError("solver terminated inside the benchmark window")

    dev.save_state()   # snapshot of the initial point (restart target of long windows)
    run_bodies(args.warmup)

    def barrier_sync():
        dev.synchronize()
        if dist is not None:
            dist.barrier()

    # the SCHUR stage (the roofline kernels) is timed inside the timed region: the library's
    # timing mode 2 stamps the 100 MHz device clock at the first workgroup start and the last
    # workgroup end of each of its launches inside the replayed graph (synchronous loop only)
    schur_live = [0.0, 0]
    if not pipelined and not os.environ.get("CLRSDP_BENCH_NO_LIVE"):
        dev.set_timing(2)
        step_plain = step

        def step():
            st = step_plain()
            schur_live[0] += st.phase_ms[_lib.STAGE_SCHUR]
            schur_live[1] += 1
            return st
        run_bodies(1)   # (re)capture the graph with the events outside the timed region
        schur_live[:] = [0.0, 0]
    barrier_sync()
    restarts.update(period=0, mu_floor=0)
    t0 = time.perf_counter()
    run_bodies(args.steps)
    barrier_sync()
    dt = time.perf_counter() - t0
    timed_restarts = dict(restarts)
    if schur_live[1]:
        step = step_plain
        dev.set_timing(False)
    # instrumented pass (per-stage HIP events, no graph replay) for the phase breakdown and the
    # Schur-assembly roofline; not part of the timed region above
    dev.set_timing(True)
    n_inst = max(3, min(args.steps, 10))
    schur_ms = 0.0
    phase = np.zeros(_lib.NUM_STAGES)
    inner = np.zeros(_lib.NUM_INNER)
    for _ in range(n_inst):
        st = step()
        ph = np.array(st.phase_ms[:])
        phase += ph
        inner += np.array(st.inner_ms[:])
        schur_ms += ph[_lib.STAGE_SCHUR]
    barrier_sync()
    dev.set_timing(False)
    # host cost of enqueueing one loop body eagerly (launch by launch, no graph: the sharded
    # path's default), i.e. the host time inside clrsdp_iterate_async; from the initial point,
    # after the timed region
    dev.restore_state()
    barrier_sync()
    dev.set_graph(False)
    enq, body = [], []
    for _ in range(12):
        t1 = time.perf_counter()
        dev.iterate_async(prm)
        t2 = time.perf_counter()
        dev.iterate_wait()
        body.append(time.perf_counter() - t1)
        enq.append(t2 - t1)
    # back to the library's own default for this handle (the graph at fp64 unless
    # CLRSDP_NO_GRAPH; eager at double-double / quad-double unless CLRSDP_GRAPH_MW)
    dev.set_graph(not env_on("CLRSDP_NO_GRAPH") and (args.precision == 1 or env_on("CLRSDP_GRAPH_MW")))
    host_enqueue_ms = float(np.median(enq[2:])) * 1e3
    eager_body_ms = float(np.median(body[2:])) * 1e3
    barrier_sync()
    if dist is not None:
        dt = dist.max_over_ranks(dt)
        schur_ms = dist.max_over_ranks(schur_ms)
        host_enqueue_ms = dist.max_over_ranks(host_enqueue_ms)
        eager_body_ms = dist.max_over_ranks(eager_body_ms)
    xranks, xbackend = dev.comm_info()

    if rank != 0:
        dev.close()   # the RCCL communicator goes with the handle, before the control plane
        dist.close()
        return
    its = args.steps / dt
    value = its   # the instance's loop bodies per second: the whole job's throughput
    fl, by = schur_flops_bytes(bi, 8 * args.precision)
    if world > 1:
        fl /= world   # per-rank share of the Schur work (the roofline is per GPU)
        by /= world
    sch_s = schur_ms / 1e3 / n_inst
    schur_src = "instrumented pass (per-stage events, no graph)"
    if schur_live[1] and schur_live[0] > 0.0:   # (the clock stamps exist on the fused fp64 path)
        sch_s = schur_live[0] / 1e3 / schur_live[1]
        schur_src = ("device clock (s_memrealtime): the sum over the SCHUR launches (at C3 the "
                     "one schur_fused_f64 launch; otherwise the V^T X^-1 and V^T Y GEMMs and the "
                     "pairs) of first workgroup start to last workgroup end, inside the replayed "
                     "graph, averaged over the timed region")
    traffic, traffic_src = schur_pmc_traffic(args.config, args.precision, world, args.clusters)
    issued, issued_src = schur_pmc_issued(args.config, args.precision, world, args.clusters)
    achieved = fl / sch_s / 1e12   # in flops of the word type (multi-word flops when w > 1)
    peak = FP64_MFMA_PEAK_TFLOPS if args.precision == 1 else MW_VALU_PEAK_TFLOPS[args.precision]
    # the library takes the int8 (Ozaki) Schur products at double-double when every block has
    # m = 1 (clrsdp.hip build_ozaki) unless CLRSDP_OZAKI=0
    ozaki = (args.precision == 2 and not os.environ.get("CLRSDP_OZAKI", "1").startswith("0")
             and all(mj == 1 for mj in bi.m))
    if ozaki:
        peak = OZAKI_DD_PEAK_TFLOPS
    # the library's default (clrsdp.hip use_graph / graph_ok): replay at world 1 unless
    # CLRSDP_NO_GRAPH, and at double-double / quad-double only with CLRSDP_GRAPH_MW; sharded only
    # with CLRSDP_GRAPH_RCCL on the native exchange
    graph_on = (not env_on("CLRSDP_NO_GRAPH")
                and (args.precision == 1 or env_on("CLRSDP_GRAPH_MW"))
                and (world == 1 or (getattr(dist, "backend", "") == "rccl"
                                    and env_on("CLRSDP_GRAPH_RCCL"))))
    res = {
        "metric": "interior-point iterations/sec (solverank1sdp loop body, MPMP.jl:755-887)",
        "value": value,
        "unit": "iterations/s",
        "instance_iterations_per_s": its,
        "shard_iterations_per_s_summed": its * world if weak else None,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": DTYPES[args.precision],
        "data": "synthetic (seeded splitmix64 instance, SURVEY.md §8d)",
        "config": {"workload": (f"{args.config}: J={cfg['J']} clusters, {cfg['delta']}x{cfg['delta']} blocks, "
                                f"rank {cfg['rank']}, N={2 * cfg['delta'] - 1} samples, n_y={cfg['n_y']}")
                               if "J" in cfg else
                               f"{args.config}: sphere-packing shape, J={bi.J} clusters, blocks "
                               f"{bi.Y_blocksizes}, dim_S {bi.dim_S}, n_y={bi.n_y}",
                   "parallelism": (f"{cfg['J'] // world} clusters per GPU on {world} GPUs (weak: one "
                                   f"C3-sized shard per GPU)" if weak else
                                   f"{cfg['J']} clusters sharded over {world} GPUs (strong)")
                                  if world > 1 else "1 GPU"},
        "roofline": {"bound": "mfma" if args.precision == 1 or ozaki else "valu",
                     "kernel": "Schur assembly (stage SCHUR)",
                     "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "peak_source": "MI355X fp64 matrix spec" if args.precision == 1 else
                                    ("int8 matrix cores (Ozaki scheme): 5.0 POPS dense / %d int8 "
                                     "multiply-adds per double-double multiply-add, in dd flops"
                                     % OZAKI_DIGIT_PAIRS) if ozaki else
                                    "measured %s multiply-add ceiling x 2 (profiles/r01_mw_peak.log)"
                                    % DTYPES[args.precision],
                     "frac": achieved / peak,
                     "issued_frac": issued, "issued_frac_source": issued_src,
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "alg_bytes_per_iteration": by,
                     "schur_ms_per_iteration": sch_s * 1e3,
                     "schur_time_source": schur_src,
                     "schur_alg_gbs": by / sch_s / 1e9},
        "phase_ms_per_iteration": {n: float(v / n_inst) for n, v in zip(_lib.STAGE_NAMES, phase)},
        # the reference's inner buckets (MPMP.jl:997-1012), same instrumented pass
        "inner_ms_per_iteration": {n: float(v / n_inst) for n, v in zip(_lib.INNER_NAMES, inner)},
        "graph_replay": graph_on,
        "exchange": "none (1 GPU)" if dist is None else dist.backend,
        # the communicator the library's loop body really uses: ranks from ncclCommCount on the
        # native RCCL path (clrsdp_comm_info), world_size on the callback path
        "exchange_ranks": xranks,
        "exchange_backend_native": xbackend,
        "host_enqueue_ms": host_enqueue_ms,
        "host_enqueue_source": ("median host time of clrsdp_iterate_async with the graph off "
                                "(clrsdp_set_graph(0): the ~100 launches of one loop body enqueued "
                                "eagerly, as the sharded path does), 10 bodies from the initial point"),
        "eager_body_ms": eager_body_ms,
        # restarts from the post-warm-up snapshot inside the timed window, by cause: every
        # RESTART = 64 bodies, or once the last body's mu fell below MU_FLOOR = 1e-8 (the
        # stagnation regime); every timed step is still one full loop body
        "restarts": {"period": timed_restarts["period"], "mu_floor": timed_restarts["mu_floor"],
                     "period_every": RESTART, "mu_floor_below": MU_FLOOR},
        "host_loop": ("pipelined (host one loop body behind, device-side pd_feas/terminate)"
                      if pipelined else
                      "synchronous (one hipGraph replay per loop body)" if graph_on else
                      "synchronous (loop body enqueued eagerly: the multi-word default)"),
    }
    if world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(pk, cons, b, bi, args.precision)
    print(json.dumps(res), flush=True)
    dev.close()
    if dist is not None:
        dist.close()


if __name__ == "__main__":
    main()
