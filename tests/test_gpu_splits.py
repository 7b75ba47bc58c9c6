"""The resident kernels the 2 / 4 / 8-GPU runs select, run with two ranks on
ONE GPU through the device exchange, at the production split's load.

A 2/4/8-GPU run of the north-star grid gives every GPU a smaller slab than
the single-GPU bench, so its Arnoldi steps run on different resident kernels
(tests/test_res_plan.py pins which): k_mgs_res<12, 0> ("pairs", 4096^2 / 8),
k_mgs_res<12, 18> ("pairs+lds", 4096^2 / 4, and with non-temporal column
loads 4096^2 / 2 and 8192^2 / 8).  Here two ranks share one GPU, each with
128 workgroups (GK_TUNE_RES_SHARE 2, resident forced on: GK_TUNE_RES 1), on a
grid chosen so that every workgroup holds the same number of register / LDS
chunks as in the production split -- the same kernel instantiation, the same
chunk loop trip counts, the in-launch cross-rank totals of
gmres_mgsr.f90:346-350's all-reduce through the exchange regions.

Check: one GMRES(95) cycle (MGS-R and Householder) against a single-context
run of the same grid -- cycle-1 true residual to 1e-9, final_err(1:95) to
1e-6, x to 1e-9 (tolerances of tests/test_gpu_configs.py; the two runs differ
only in the dot-product summation order), every rank taking the same decisions.
"""
import multiprocessing as mp
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M = 95
# grid, expected variant, forced NT (None: auto), the production split it stands for
CASES = [
    (1448, "pairs", None, "4096^2 on 8 GPUs"),
    (2048, "pairs+lds", None, "4096^2 on 4 GPUs"),
    (2896, "pairs+lds", 1, "4096^2 on 2 GPUs, 8192^2 on 8 GPUs"),
    (4096, "w-only", None, "4096^2 on 1 GPU (per-workgroup load)"),
]


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


def _tune_forced(c, nt):
    from gmres_amd import _native as nat

    c.tune(nat.GK_TUNE_RES, 1)
    c.tune(nat.GK_TUNE_RES_SHARE, 2)
    c.tune(nat.GK_TUNE_RES_TIMEOUT_MS, 10000)
    c.tune(nat.GK_TUNE_XCHG_TIMEOUT_MS, 10000)
    if nt is not None:
        c.tune(nat.GK_TUNE_PROJ_NT, nt)


def _compare(ref, res, xs):
    assert len({(r.n_out, r.cycles_out, r.n_cycles) for r in res}) == 1
    assert all(np.array_equal(res[0].hist_res, r.hist_res) for r in res)
    assert all(np.array_equal(res[0].final_err, r.final_err) for r in res)
    assert res[0].n_out == M
    assert res[0].hist_res[0] == pytest.approx(ref.hist_res[0], rel=1e-9)
    assert np.allclose(res[0].final_err[:M], ref.final_err[:M], rtol=1e-6, atol=0)
    assert np.allclose(np.concatenate(xs), ref.x, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("method", ["mgsr", "hh"])
@pytest.mark.parametrize("N,variant,nt,prod", CASES)
def test_split_variant_two_ranks_in_process(N, variant, nt, prod, method):
    import gmres_amd as ga

    ref = _single(N, method)
    parts = ga.slab_partition(N, 2)
    g = ga.LocalGroup(2)
    ctxs = [ga.Context(N, M, device=0, line0=l0, nlines=nl) for l0, nl in parts]
    out, err = [None, None], []
    try:
        for r, c in enumerate(ctxs):
            c.comm_init_local(g, r, max(nl for _, nl in parts))
        for c in ctxs:
            c.xchg_local()
            _tune_forced(c, nt)
        plans = [c.res_info(hh=(method == "hh")) for c in ctxs]
        assert all(p["variant"] == variant and p["G"] == 128 for p in plans), (prod, plans)

        def work(r):
            try:
                c = ctxs[r]
                c.set_rhs_ones()
                c.profile(True)
                c.profile_reset()
                out[r] = (_solve(c, method), c.profile_read())
            except Exception as e:  # pragma: no cover - reported below
                err.append(e)

        th = [threading.Thread(target=work, args=(r,)) for r in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=110)
        assert not err, err
        assert all(o is not None for o in out)
        # every Arnoldi step ran as a resident launch (no launch-per-projection fallback)
        assert all(o[1]["res"][1] >= M for o in out)
        _compare(ref, [o[0] for o in out], [o[0].x for o in out])
    finally:
        for c in ctxs:
            c.close()
        g.close()


# ------------------------------------------------ two processes (IPC) ------

def _ipc_worker(rank, N, nt, hq, hin, outq, done):
    try:
        import gmres_amd as ga

        parts = ga.slab_partition(N, 2)
        l0, nl = parts[rank]
        c = ga.Context(N, M, device=0, line0=l0, nlines=nl)
        c.comm_init_xgmi(2, rank, max(n for _, n in parts))
        hq.put((rank, c.xchg_handle()))
        c.xchg_open(hin.get(timeout=100))
        _tune_forced(c, nt)
        if not c.xchg_selftest(10000):
            outq.put((rank, "selftest", c.xchg_error))
        else:
            plan = c.res_info()
            c.set_rhs_ones()
            c.profile(True)
            c.profile_reset()
            r = _solve(c, "mgsr")
            prof = c.profile_read()
            outq.put((rank, "ok", (plan, prof["res"][1], r.hist_res, r.final_err, r.n_out, r.x)))
        done.wait(120)  # keep the exchange region mapped until the peer is done with it
        c.close()
    except Exception as e:  # pragma: no cover - reported to the parent
        outq.put((rank, "error", repr(e)))


@pytest.mark.parametrize("N,variant,nt,prod", [CASES[0], CASES[2]])
def test_split_variant_two_processes_ipc(N, variant, nt, prod):
    """The same as above with the ranks in two processes sharing their exchange
    regions by IPC handles: the transport of the multi-GPU bench."""
    ref = _single(N, "mgsr")
    ctx = mp.get_context("spawn")
    hq, outq, done = ctx.Queue(), ctx.Queue(), ctx.Event()
    hins = [ctx.Queue() for _ in range(2)]
    ps = [ctx.Process(target=_ipc_worker, args=(r, N, nt, hq, hins[r], outq, done)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        hs = dict(hq.get(timeout=100) for _ in range(2))
        for q in hins:
            q.put([hs[0], hs[1]])
        got = dict((r, (kind, val)) for r, kind, val in (outq.get(timeout=110) for _ in range(2)))
    finally:
        done.set()
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(2):
        assert got[r][0] == "ok", got[r]
    vals = [got[r][1] for r in range(2)]
    assert all(v[0]["variant"] == variant and v[0]["G"] == 128 for v in vals), (prod, [v[0] for v in vals])
    assert all(v[1] >= M for v in vals)  # every Arnoldi step a resident launch
    assert np.array_equal(vals[0][2], vals[1][2]) and np.array_equal(vals[0][3], vals[1][3])
    assert vals[0][4] == M
    assert vals[0][2][0] == pytest.approx(ref.hist_res[0], rel=1e-9)
    assert np.allclose(vals[0][3][:M], ref.final_err[:M], rtol=1e-6, atol=0)
    assert np.allclose(np.concatenate([vals[0][5], vals[1][5]]), ref.x, rtol=1e-9, atol=1e-12)
