"""The resident kernels the 2 / 4 / 8-GPU runs select, run with 2, 4 and 8
ranks on ONE GPU through the device exchange, at the production split's load.

A 2/4/8-GPU run of the north-star grid gives every GPU a smaller slab than
the single-GPU bench, so its Arnoldi steps run on different resident kernels
(tests/test_res_plan.py pins which): k_mgs_res<8, 0> ("pairs", 4096^2 / 8),
k_mgs_res<12, 4> ("pairs+lds", 4096^2 / 4) and the column-cache kernel k_mgs_wpc
("w+column": w in registers, the running Krylov column cached in registers +
LDS; 4096^2 / 2 and 8192^2 / 8).  Here R ranks share
one GPU, each with 256 / R workgroups (GK_TUNE_RES_SHARE R, resident forced
on: GK_TUNE_RES 1), on a grid chosen so that every workgroup holds the same
number of register / LDS chunks as in the production split -- the same kernel
instantiation, the same chunk loop trip counts -- and the in-launch
cross-rank totals of gmres_mgsr.f90:346-350's all-reduce run with R rank
totals (workgroup 0 of every rank pushes its total into 8 replicated slots of
every peer's region; every workgroup sums the R totals in rank order).  With
256 / R workgroups per rank the same grid N^2 carries the same load for every
R: 1448^2 ~ 4096^2 / 8, 2048^2 ~ 4096^2 / 4, 2896^2 ~ 4096^2 / 2 and
8192^2 / 8, 4096^2 ~ the single-GPU bench.

Check: one GMRES(95) cycle (MGS-R and Householder) against a single-context
run of the same grid AND against the reference's own cycle 1 at that grid
(round 5 fixtures: the cycle-1 true residual to 1e-9; round 6: the reference's
full cycle 1 -- final_err(1:95) to 1e-9 and x sampled every 4099th unknown to
1e-9) -- against the single context: final_err(1:95) to 1e-6, x to 1e-9 (tolerances of tests/test_gpu_configs.py; the two runs differ
only in the dot-product summation order) -- with the selected variant and
workgroup count asserted, every Arnoldi step a resident launch, no
launch-per-projection all-reduce, and every rank taking the same decisions.
"""
import multiprocessing as mp
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M = 95
# grid, expected variant, the production split it stands for
CASES = [
    (1448, "pairs", "4096^2 on 8 GPUs"),
    (2048, "w+column", "4096^2 on 4 GPUs"),
    (2896, "w+column", "4096^2 on 2 GPUs, 8192^2 on 8 GPUs"),
    (4096, "w-only", "4096^2 on 1 GPU (per-workgroup load)"),
]
PROD = {1448: (4096, 8), 2048: (4096, 4), 2896: (4096, 2), 4096: (4096, 1)}


def _prod_nt(N):
    """The column load policy the production split selects (non-temporal once
    its slab outgrows the Infinity Cache): forced on the test grid, whose
    smaller slab would pick the other policy by itself."""
    import gmres_amd as ga

    PN, PR = PROD[N]
    nl = max(n for _, n in ga.slab_partition(PN, PR))
    return ga.res_plan_query(PN * nl, 256, 1, False, -1)["nt"]


def _single(N, method):
    import gmres_amd as ga

    with ga.Context(N, M) as c:
        c.set_rhs_ones()
        r = _solve(c, method)
        return r


def _solve(c, method):
    import gmres_amd as ga

    if method == "mgsr":
        return ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False, want_hist=True)
    return ga.gmres_hh(c, 1e-15, precondition=False, max_cycles=1, want_verr=False, want_hist=True)


def _tune_forced(c, nt, R):
    from gmres_amd import _native as nat

    c.tune(nat.GK_TUNE_RES, 1)
    c.tune(nat.GK_TUNE_RES_SHARE, R)
    c.tune(nat.GK_TUNE_RES_TIMEOUT_MS, 10000)
    c.tune(nat.GK_TUNE_XCHG_TIMEOUT_MS, 10000)
    c.tune(nat.GK_TUNE_PROJ_NT, nt)


def _ref_cycle1(N, method):
    """The REFERENCE's own cycle-1 true residual at this grid (oracle/_ref, 8
    threads; tests/golden/make_ref_fixtures.py, round 5 for 1448^2 / 2048^2 /
    2896^2) -- gmres_mgsr.f90:309-413, gmres_hh.f90:211-385."""
    import json
    import os

    runs = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_runs.json")))
    return runs[f"{method}_omp_identity_{N}_m95_1cyc_t8"]["hist_res"][0]


def _ref_full_cycle1(N, method):
    """The REFERENCE's cycle 1 in full at this grid (round 6): final_err(1:95) and x
    sampled every x_stride-th unknown, from a run whose tol ends it after exactly one
    full cycle (tests/golden/make_ref_fixtures.py SPLIT_FE); None before those exist."""
    import json
    import os

    runs = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_runs.json")))
    return runs.get(f"{method}_omp_identity_{N}_m95_cyc1full_t8")


def _compare(ref, res, xs, N=None, method=None):
    assert len({(r.n_out, r.cycles_out, r.n_cycles) for r in res}) == 1
    assert all(np.array_equal(res[0].hist_res, r.hist_res) for r in res)
    assert all(np.array_equal(res[0].final_err, r.final_err) for r in res)
    assert res[0].n_out == M
    assert res[0].hist_res[0] == pytest.approx(ref.hist_res[0], rel=1e-9)
    assert np.allclose(res[0].final_err[:M], ref.final_err[:M], rtol=1e-6, atol=0)
    x = np.concatenate(xs)
    assert np.allclose(x, ref.x, rtol=1e-9, atol=1e-12)
    if N is not None:  # rank 0's cycle 1 against the reference's own run, not only HIP's
        assert res[0].hist_res[0] == pytest.approx(_ref_cycle1(N, method), rel=1e-9)
        g = _ref_full_cycle1(N, method)
        if g is not None:  # final_err(1:95) and x (sampled) of the reference's full cycle 1
            assert np.allclose(res[0].final_err[:M], g["final_err"], rtol=1e-9, atol=0)
            assert np.allclose(x[:: g["x_stride"]], g["x_sample"], rtol=1e-9, atol=1e-12)


def _check_profile(outs, method):
    """Every Arnoldi step ran as resident launches (MGS-R: one per step; HH: the
    two chains of every step) and no projection went through a per-projection
    launch or an all-reduce call -- the rank totals travelled inside the launches
    (the only collective calls left are the cycle start's all-reduce of the
    norm and, for HH, the broadcasts of the H column)."""
    for prof in outs:
        assert prof["res"][1] >= (M if method == "mgsr" else 2 * M), prof
        assert prof["proj"][1] <= 1, prof  # the solve's ||b|| (gmres_mgsr.f90:307), never a projection


@pytest.mark.parametrize("method", ["mgsr", "hh"])
@pytest.mark.parametrize("R", [2, 4, 8])
@pytest.mark.parametrize("N,variant,prod", CASES)
def test_split_variant_in_process(N, variant, prod, R, method):
    import gmres_amd as ga

    nt = _prod_nt(N)
    ref = _single(N, method)
    parts = ga.slab_partition(N, R)
    g = ga.LocalGroup(R)
    ctxs = [ga.Context(N, M, device=0, line0=l0, nlines=nl) for l0, nl in parts]
    out, err = [None] * R, []
    try:
        for r, c in enumerate(ctxs):
            c.comm_init_local(g, r, max(nl for _, nl in parts))
        for c in ctxs:
            c.xchg_local()
            _tune_forced(c, nt, R)
        plans = [c.res_info(hh=(method == "hh")) for c in ctxs]
        assert all(p["variant"] == variant and p["G"] == 256 // R for p in plans), (prod, plans)
        assert len({(p["r2e"], p["l2e"], p["nt"]) for p in plans}) == 1, plans

        def work(r):
            try:
                c = ctxs[r]
                c.set_rhs_ones()
                c.profile(True)
                c.profile_reset()
                out[r] = (_solve(c, method), c.profile_read())
            except Exception as e:  # pragma: no cover - reported below
                err.append(e)

        th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=110)
        assert not err, err
        assert all(o is not None for o in out)
        _check_profile([o[1] for o in out], method)
        _compare(ref, [o[0] for o in out], [o[0].x for o in out], N, method)
    finally:
        for c in ctxs:
            c.close()
        g.close()


@pytest.mark.parametrize("method", ["mgsr", "hh"])
@pytest.mark.parametrize("N,variant", [(1448, "pairs"), (2048, "w+column"), (2896, "w+column")])
def test_first_dot_fold(N, variant, method):
    """GK_TUNE_RES_FOLD: on 2 ranks the MGS step's first dot <w, V(:,1)> (the
    Householder step's <w, P_1>) is summed
    across ranks inside the resident launch (each rank's partial slab summed
    locally, then the rank-total hop) instead of by a k_xchg launch before it --
    one collective launch fewer per Arnoldi step, the same cycle up to the
    summation order of that one dot."""
    import gmres_amd as ga
    from gmres_amd import _native as nat

    R, nt = 2, _prod_nt(N)
    parts = ga.slab_partition(N, R)
    runs = {}
    for fold in (0, 1):
        g = ga.LocalGroup(R)
        ctxs = [ga.Context(N, M, device=0, line0=l0, nlines=nl) for l0, nl in parts]
        out, err = [None] * R, []
        try:
            for r, c in enumerate(ctxs):
                c.comm_init_local(g, r, max(nl for _, nl in parts))
            for c in ctxs:
                c.xchg_local()
                _tune_forced(c, nt, R)
                c.tune(nat.GK_TUNE_RES_FOLD, fold)
            assert all(c.res_info(hh=(method == "hh"))["variant"] == variant for c in ctxs)

            def work(r):
                try:
                    c = ctxs[r]
                    c.set_rhs_ones()
                    c.profile(True)
                    c.profile_reset()
                    out[r] = (_solve(c, method), c.profile_read())
                except Exception as e:  # pragma: no cover - reported below
                    err.append(e)

            th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=110)
            assert not err, err
            assert all(o is not None for o in out)
            runs[fold] = out
        finally:
            for c in ctxs:
                c.close()
            g.close()
    (r0, p0), (r1, p1) = runs[0][0], runs[1][0]
    assert all(np.array_equal(r1.hist_res, o[0].hist_res) for o in runs[1])  # every rank the same decisions
    assert r1.n_out == r0.n_out == M
    assert r1.hist_res[0] == pytest.approx(r0.hist_res[0], rel=1e-12)
    assert np.allclose(r1.final_err[:M], r0.final_err[:M], rtol=1e-9, atol=0)
    # one all-reduce launch fewer per Arnoldi step
    assert p0["comm"][1] - p1["comm"][1] == M, (p0["comm"], p1["comm"])
    assert p1["res"][1] == p0["res"][1] >= (M if method == "mgsr" else 2 * M)


# ------------------------------------------------ two processes (IPC) ------

def _ipc_worker(rank, R, N, nt, method, hq, hin, outq, done):
    try:
        import gmres_amd as ga

        parts = ga.slab_partition(N, R)
        l0, nl = parts[rank]
        c = ga.Context(N, M, device=0, line0=l0, nlines=nl)
        c.comm_init_xgmi(R, rank, max(n for _, n in parts))
        hq.put((rank, c.xchg_handle()))
        c.xchg_open(hin.get(timeout=100))
        _tune_forced(c, nt, R)
        if not c.xchg_selftest(10000):
            outq.put((rank, "selftest", c.xchg_error))
        else:
            plan = c.res_info(hh=(method == "hh"))
            c.set_rhs_ones()
            c.profile(True)
            c.profile_reset()
            r = _solve(c, method)
            prof = c.profile_read()
            outq.put((rank, "ok", (plan, prof, r.hist_res, r.final_err, r.n_out, r.x, ga.runtime_info())))
        done.wait(120)  # keep the exchange region mapped until every peer is done with it
        c.close()
    except Exception as e:  # pragma: no cover - reported to the parent
        outq.put((rank, "error", repr(e)))


@pytest.mark.parametrize("R,N,variant,prod,method", [
    (2, *CASES[0], "mgsr"), (2, *CASES[2], "mgsr"),
    (4, *CASES[1], "mgsr"), (4, *CASES[2], "hh"),
])
def test_split_variant_processes_ipc(R, N, variant, prod, method):
    """The same with the ranks in R processes sharing their exchange regions by
    IPC handles: the transport of the multi-GPU bench.  The workers never import
    torch, so they run on the HIP runtime / RCCL the library was built against."""
    ref = _single(N, method)
    nt = _prod_nt(N)
    ctx = mp.get_context("spawn")
    hq, outq, done = ctx.Queue(), ctx.Queue(), ctx.Event()
    hins = [ctx.Queue() for _ in range(R)]
    ps = [ctx.Process(target=_ipc_worker, args=(r, R, N, nt, method, hq, hins[r], outq, done)) for r in range(R)]
    for p in ps:
        p.start()
    try:
        hs = dict(hq.get(timeout=100) for _ in range(R))
        for q in hins:
            q.put([hs[r] for r in range(R)])
        got = dict((r, (kind, val)) for r, kind, val in (outq.get(timeout=110) for _ in range(R)))
    finally:
        done.set()
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(R):
        assert got[r][0] == "ok", got[r]
    vals = [got[r][1] for r in range(R)]
    assert all(v[0]["variant"] == variant and v[0]["G"] == 256 // R for v in vals), \
        (prod, [v[0] for v in vals])
    _check_profile([v[1] for v in vals], method)
    assert all(np.array_equal(vals[0][2], v[2]) and np.array_equal(vals[0][3], v[3]) for v in vals)
    assert vals[0][4] == M
    assert vals[0][2][0] == pytest.approx(ref.hist_res[0], rel=1e-9)
    assert vals[0][2][0] == pytest.approx(_ref_cycle1(N, method), rel=1e-9)
    assert np.allclose(vals[0][3][:M], ref.final_err[:M], rtol=1e-6, atol=0)
    assert np.allclose(np.concatenate([v[5] for v in vals]), ref.x, rtol=1e-9, atol=1e-12)
    rt = vals[0][6]  # torch-free workers: the runtime the library links, not torch's bundled one
    assert not rt["torch_imported"] and "/torch/" not in (rt["libamdhip64"] or ""), rt
