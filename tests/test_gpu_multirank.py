"""Multi-rank slab decomposition on ONE GPU: 2-4 contexts (one host thread
each) joined by the in-process communicator (gk_group), which replays the
RCCL message pattern of the multi-GPU path -- halo lines before every stencil
sweep, all-reduced partial slabs, the Householder pivot broadcast, the Gram
all-reduce -- on the real HIP kernels and the replicated Fortran host loops.
The concatenated result must match the single-context solve."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _single(N, m, method, prec, degree, max_cycles, res=-1):
    import gmres_amd as ga

    with ga.Context(N, m) as c:
        c.tune(8, res)  # GK_TUNE_RES: -1 auto; 0 = the launch-per-projection path
        c.set_precond(prec, (8.2, 0.2), degree)
        c.set_rhs_ones()
        return _solve(c, method, prec, max_cycles)


def _solve(c, method, prec, max_cycles):
    import gmres_amd as ga

    if method == "mgsr":
        return ga.gmres_mgsr(c, 1e-15, max_cycles=max_cycles, want_hist=True)
    return ga.gmres_hh(c, 1e-15, precondition=(prec != "identity"), max_cycles=max_cycles, want_hist=True)


def _group(N, m, nranks, method, prec, degree, max_cycles):
    import gmres_amd as ga

    parts = ga.slab_partition(N, nranks)
    ml = max(nl for _, nl in parts)
    g = ga.LocalGroup(nranks)
    ctxs = [ga.Context(N, m, device=0, line0=l0, nlines=nl) for l0, nl in parts]
    for r, c in enumerate(ctxs):
        c.comm_init_local(g, r, ml)
    out = [None] * nranks
    err = []

    def work(r):
        try:
            c = ctxs[r]
            c.set_precond(prec, (8.2, 0.2), degree)
            c.set_rhs_ones()
            out[r] = _solve(c, method, prec, max_cycles)
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not err, err
    for c in ctxs:
        c.close()
    g.close()
    return out


@pytest.mark.parametrize("nranks", [2, 3, 4])
@pytest.mark.parametrize("method,prec,degree", [("mgsr", "identity", 1), ("mgsr", "cbpr2", 1), ("mgsr", "cheb", 4),
                                                ("hh", "identity", 1), ("hh", "cbpr2", 1)])
def test_slabs_match_single_context(nranks, method, prec, degree):
    N, m, cyc = 66, 16, 6
    ref = _single(N, m, method, prec, degree, cyc)
    res = _group(N, m, nranks, method, prec, degree, cyc)
    # replicated host loops: every rank took the same decisions
    assert len({(r.n_out, r.cycles_out, r.n_cycles) for r in res}) == 1
    assert np.array_equal(res[0].hist_res, res[-1].hist_res)
    x = np.concatenate([r.x for r in res])
    k = min(len(ref.hist_res), len(res[0].hist_res))
    h, rr = res[0].hist_res[:k], ref.hist_res[:k]
    # MGS-R: 1e-3 below r = 1e-6; Householder: the tiers of test_gpu_solver._hist_close_hh
    tol = np.where(rr > 1e-6, 1e-9, 1e-3 if method == "mgsr" else np.where(rr > 1e-12, 1e-3, 5e-2))
    assert np.all(np.abs(h - rr) <= tol * rr + 1e-16), (h, rr)
    if ref.hist_res[-1] > 1e-6:  # still far from the floor: x itself must agree closely
        assert np.allclose(x, ref.x, rtol=1e-9, atol=1e-12)


def test_slabs_converge_and_verr():
    """Full solve to tol on 3 ranks: converges to x = 1 with a small v_err."""
    import gmres_amd as ga

    N, m = 48, 20
    res = _group(N, m, 3, "mgsr", "cbpr2", 1, 1000)
    x = np.concatenate([r.x for r in res])
    assert np.max(np.abs(x - 1.0)) < 1e-9
    assert res[0].final_err[res[0].n_out - 1] < 1e-15
    assert 0 <= res[0].v_err[res[0].n_out - 1] < 1e-12
    ref = _single(N, m, "mgsr", "cbpr2", 1, 1000)
    assert abs(res[0].iterations - ref.iterations) <= max(2, 0.01 * ref.iterations)


def test_lanczos_independent_of_decomposition():
    import gmres_amd as ga

    N = 40
    with ga.Context(N, 8) as c:
        ref = c.lanczos_bounds(30)
    parts = ga.slab_partition(N, 3)
    g = ga.LocalGroup(3)
    ctxs = [ga.Context(N, 8, line0=l0, nlines=nl) for l0, nl in parts]
    for r, c in enumerate(ctxs):
        c.comm_init_local(g, r, max(nl for _, nl in parts))
    out = [None] * 3

    def work(r):
        out[r] = ctxs[r].lanczos_bounds(30)

    th = [threading.Thread(target=work, args=(r,)) for r in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert out[0] == out[1] == out[2]
    assert out[0][0] == pytest.approx(ref[0], rel=1e-9) and out[0][1] == pytest.approx(ref[1], rel=1e-12)
    for c in ctxs:
        c.close()
    g.close()


@pytest.mark.parametrize("method,prec", [("mgsr", "cbpr2"), ("hh", "identity")])
def test_rccl_one_rank_communicator(monkeypatch, method, prec):
    """The RCCL code path on one GPU: a 1-rank communicator (GK_FORCE_RCCL=1)
    routes every slab all-reduce, broadcast and (empty) halo group through
    RCCL on the context stream; results must equal the communicator-free run
    bit for bit (a 1-rank sum is exact)."""
    import gmres_amd as ga

    N, m = 64, 16
    ref = _single(N, m, method, prec, 1, 4, res=0)  # same kernels (RCCL cannot drive the resident step)
    monkeypatch.setenv("GK_FORCE_RCCL", "1")
    with ga.Context(N, m) as c:
        c.comm_init(1, 0, N, ga.Context.unique_id())
        c.set_precond(prec, (8.2, 0.2), 1)
        c.set_rhs_ones()
        r = _solve(c, method, prec, 4)
    assert np.array_equal(r.hist_res, ref.hist_res)
    assert np.array_equal(r.x, ref.x)


@pytest.mark.parametrize("rccl", [False, True])
def test_launch_path_step_graphs(monkeypatch, rccl):
    """GK_TUNE_GRAPH: the launch-path MGS-R step (2j projection launches, 2j + 1
    all-reduces -- ncclAllReduce captured as graph nodes on the RCCL path -- and
    the normalisation) captured once per j and replayed in later cycles gives
    the call-by-call results bit for bit; the graph replays are what ran (the
    'graph' profile slot) and the per-step time is recorded for the A/B."""
    import time

    import gmres_amd as ga
    from gmres_amd import _native as nat

    N, m, cyc = 256, 30, 4
    out = {}
    for graph in (0, 1):
        if rccl:
            monkeypatch.setenv("GK_FORCE_RCCL", "1")
        with ga.Context(N, m) as c:
            if rccl:
                c.comm_init(1, 0, N, ga.Context.unique_id())
            c.tune(nat.GK_TUNE_RES, 0)
            c.tune(nat.GK_TUNE_GRAPH, graph)
            c.set_rhs_ones()
            ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)  # warm (graphs captured here)
            c.profile(True)
            c.profile_reset()
            c.sync()
            t0 = time.perf_counter()
            r = ga.gmres_mgsr(c, 1e-15, max_cycles=cyc, want_hist=True, want_verr=False)
            c.sync()
            out[graph] = (r, c.profile_read(), time.perf_counter() - t0)
    r0, p0, t0 = out[0]
    r1, p1, t1 = out[1]
    assert np.array_equal(r0.hist_res, r1.hist_res) and np.array_equal(r0.x, r1.x)
    assert np.array_equal(r0.final_err, r1.final_err)
    assert p1["graph"][1] == cyc * m and p1["proj"][1] <= 1, p1  # 1: the solve's ||b||
    assert p0["graph"][1] == 0 and p0["proj"][1] > 0, p0
    print(f"launch path {'RCCL' if rccl else 'single'} {N}^2 m={m}: {t0 / cyc * 1e3:.2f} ms/cycle call by call, "
          f"{t1 / cyc * 1e3:.2f} ms/cycle replayed graphs")


@pytest.mark.parametrize("rccl", [False, True])
def test_launch_path_capture_failure(monkeypatch, rccl):
    """A step-graph capture that fails (forced: GK_DEBUG_CAPTURE_FAIL) switches graphs
    off for a single-rank context, which then runs call by call with the same bits;
    on an RCCL rank it is an error naming the remedy (GK_TUNE_GRAPH 0 on every rank),
    since one rank running eagerly while its peers replay is not supported."""
    import gmres_amd as ga
    from gmres_amd import _native as nat

    N, m = 256, 30
    if rccl:
        monkeypatch.setenv("GK_FORCE_RCCL", "1")

    def run(fail):
        if fail:
            monkeypatch.setenv("GK_DEBUG_CAPTURE_FAIL", "1")
        else:
            monkeypatch.delenv("GK_DEBUG_CAPTURE_FAIL", raising=False)
        with ga.Context(N, m) as c:
            if rccl:
                c.comm_init(1, 0, N, ga.Context.unique_id())
            c.tune(nat.GK_TUNE_RES, 0)
            c.tune(nat.GK_TUNE_GRAPH, 1)
            c.set_rhs_ones()
            return ga.gmres_mgsr(c, 1e-15, max_cycles=2, want_hist=True, want_verr=False)

    ref = run(False)
    if rccl:
        with pytest.raises(ga.GkError, match="GK_TUNE_GRAPH 0"):
            run(True)
    else:
        r = run(True)
        assert np.array_equal(r.hist_res, ref.hist_res) and np.array_equal(r.x, ref.x)


@pytest.mark.parametrize("R", [2, 3])
def test_launch_path_step_graphs_device_exchange(R):
    """GK_TUNE_GRAPH over the device exchange (in-process slab ranks, resident
    kernels off): the captured step's k_xchg launches read their sequence
    numbers from a device base the host sets before every replay, so replayed
    graphs keep the exchange's numbering -- results equal the call-by-call run
    bit for bit on every rank, and every Arnoldi step ran as a replay."""
    import time

    import gmres_amd as ga
    from gmres_amd import _native as nat

    N, m, cyc = 256, 30, 4
    parts = ga.slab_partition(N, R)
    runs = {}
    for graph in (0, 1):
        g = ga.LocalGroup(R)
        ctxs = [ga.Context(N, m, device=0, line0=l0, nlines=nl) for l0, nl in parts]
        out, err = [None] * R, []
        try:
            for r, c in enumerate(ctxs):
                c.comm_init_local(g, r, max(nl for _, nl in parts))
            for c in ctxs:
                c.xchg_local()
                c.tune(nat.GK_TUNE_RES, 0)
                c.tune(nat.GK_TUNE_GRAPH, graph)

            def work(r):
                try:
                    c = ctxs[r]
                    c.set_rhs_ones()
                    ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)  # graphs captured here
                    c.profile(True)
                    c.profile_reset()
                    c.sync()
                    t0 = time.perf_counter()
                    res = ga.gmres_mgsr(c, 1e-15, max_cycles=cyc, want_hist=True, want_verr=False)
                    c.sync()
                    out[r] = (res, c.profile_read(), time.perf_counter() - t0)
                except Exception as e:  # pragma: no cover - reported below
                    err.append(e)

            th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=100)
            assert not err, err
            assert all(o is not None for o in out)
            runs[graph] = out
        finally:
            for c in ctxs:
                c.close()
            g.close()
    for r in range(R):
        r0, p0, _ = runs[0][r]
        r1, p1, _ = runs[1][r]
        assert np.array_equal(r0.hist_res, r1.hist_res) and np.array_equal(r0.x, r1.x)
        assert p1["graph"][1] == cyc * m and p1["proj"][1] <= 1, p1
        assert p0["graph"][1] == 0 and p0["proj"][1] > 0, p0
    t0 = max(o[2] for o in runs[0]) / cyc * 1e3
    t1 = max(o[2] for o in runs[1]) / cyc * 1e3
    print(f"launch path, device exchange, {R} ranks {N}^2 m={m}: {t0:.2f} ms/cycle call by call, "
          f"{t1:.2f} ms/cycle replayed graphs")


@pytest.mark.parametrize("N,nranks", [(66, 3), (20, 4), (16, 5), (130, 2)])
@pytest.mark.parametrize("degree", [1, 3, 4, 6, 8])
def test_chebyshev_on_slabs_bitexact(oracle, N, nranks, degree):
    """M^-1 r on row-block slabs: the temporal-blocked Chebyshev pass (one pass
    of L = k <= 8 levels) takes a deep halo (L lines of its input from each
    neighbour) and gives the single-grid result bit for bit; when any slab is
    thinner than L lines (16 / 5 at degree >= 4, 20 / 4 at degree 6 and 8) every
    rank takes the per-sweep kernels with one-line halos, also bit-exact."""
    import gmres_amd as ga

    r = np.random.default_rng(N + degree).standard_normal(N * N)
    ref = oracle.precond(oracle.PREC_CHEB, r, N, params=(8.2, 0.2), degree=degree)
    parts = ga.slab_partition(N, nranks)
    g = ga.LocalGroup(nranks)
    ctxs = [ga.Context(N, 8, line0=l0, nlines=nl) for l0, nl in parts]
    out = [None] * nranks
    try:
        for q, c in enumerate(ctxs):
            c.comm_init_local(g, q, max(nl for _, nl in parts))
            c.set_precond("cheb", (8.2, 0.2), degree)

        def work(q):
            l0, nl = parts[q]
            out[q] = ctxs[q].apply(r[l0 * N:(l0 + nl) * N], 1)

        th = [threading.Thread(target=work, args=(q,)) for q in range(nranks)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=60)
        assert np.array_equal(np.concatenate(out), ref)
    finally:
        for c in ctxs:
            c.close()
        g.close()


def test_comm_latency_local_group_and_single():
    """gk_comm_latency through the in-process group (RCCL's message pattern),
    and zeros on a single context (no collective)."""
    import threading

    import gmres_amd as ga

    with ga.Context(32, 4) as c:
        assert c.comm_latency(10) == {"allreduce_us": 0.0, "halo_us": 0.0}
    parts = ga.slab_partition(64, 2)
    g = ga.LocalGroup(2)
    ctxs = [ga.Context(64, 8, device=0, line0=l0, nlines=nl) for l0, nl in parts]
    out = [None, None]
    try:
        for r, c in enumerate(ctxs):
            c.comm_init_local(g, r, max(nl for _, nl in parts))
        th = [threading.Thread(target=lambda r=r: out.__setitem__(r, ctxs[r].comm_latency(20))) for r in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert all(o is not None and o["allreduce_us"] > 0 and o["halo_us"] > 0 for o in out), out
    finally:
        for c in ctxs:
            c.close()
        g.close()


@pytest.mark.parametrize("transport", ["local", "xchg"])
@pytest.mark.parametrize("degree", [2, 8])
def test_chebyshev_uneven_slabs_bitexact(oracle, transport, degree):
    """Any consecutive slabs, not only slab_partition's: a 2-line slab between
    wide ones.  The temporal-blocked pass needs L lines of every neighbour, so
    the smallest slab of ANY rank (gathered once over the communicator) decides
    for all ranks together: degree 2 keeps the fused pass (2 >= L = 2), degree 8
    drops every rank to the per-sweep kernels.  Bit-exact against the oracle
    either way, through the in-process group and the device exchange."""
    import gmres_amd as ga

    N = 40
    parts = [(0, 19), (19, 2), (21, 19)]
    r = np.random.default_rng(degree).standard_normal(N * N)
    ref = oracle.precond(oracle.PREC_CHEB, r, N, params=(8.2, 0.2), degree=degree)
    g = ga.LocalGroup(3)
    ctxs = [ga.Context(N, 8, line0=l0, nlines=nl) for l0, nl in parts]
    out, err = [None] * 3, []
    try:
        for q, c in enumerate(ctxs):
            c.comm_init_local(g, q, 19)
        if transport == "xchg":
            for c in ctxs:
                c.xchg_local()
        for c in ctxs:
            c.set_precond("cheb", (8.2, 0.2), degree)

        def work(q):
            try:
                l0, nl = parts[q]
                out[q] = ctxs[q].apply(r[l0 * N:(l0 + nl) * N], 1)
            except Exception as e:  # pragma: no cover - reported below
                err.append(e)

        th = [threading.Thread(target=work, args=(q,)) for q in range(3)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=60)
        assert not err, err
        assert np.array_equal(np.concatenate(out), ref)
    finally:
        for c in ctxs:
            c.close()
        g.close()


def _arnoldi_steps(c, nsteps):
    """Cycle start + Arnoldi steps 1..nsteps through the C-ABI pieces: the H
    columns and the local slab of V(:, nsteps + 1)."""
    c.set_rhs_ones()
    beta = c.mgs_cycle_start()
    H = [c.mgs_step(j) for j in range(1, nsteps + 1)]
    return beta, H, c.get_basis(nsteps)


@pytest.mark.parametrize("transport", ["local", "xchg"])
@pytest.mark.parametrize("split", ["even2", "even3", "thin"])
@pytest.mark.parametrize("degree", [4, 8])
def test_chebyshev_stencil_stage_on_slabs(transport, split, degree):
    """The Arnoldi step's Chebyshev pass with the stencil as its stage 0
    (GK_TUNE_CHEB_STEN, N >= 128) on row-block slabs: the pass takes k + 1
    deep-halo lines of v (CF_HMAX, XS_HALO_LINES) and indexes the row + halo
    offsets itself.  N = 130, Chebyshev(4) and (8), 2 and 3 ranks, through the
    in-process group and the device exchange; 'thin' puts a slab of exactly k
    lines between wide ones, so the k + 1 gate sends EVERY rank to the stencil
    launch + pass route together.  Against one context: beta, the H columns of
    steps 1..5 and V(:,6) (dot-product summation order only)."""
    import gmres_amd as ga

    N, m, steps = 130, 8, 5
    with ga.Context(N, m) as c:
        c.set_precond("cheb", (8.2, 0.2), degree)
        b0, H0, v0 = _arnoldi_steps(c, steps)
        assert c.res_info()["cheb_sten"] == 1
    if split == "thin":
        w = (N - degree) // 2
        parts = [(0, w), (w, degree), (w + degree, N - w - degree)]
    else:
        parts = ga.slab_partition(N, 2 if split == "even2" else 3)
    R = len(parts)
    g = ga.LocalGroup(R)
    ctxs = [ga.Context(N, m, device=0, line0=l0, nlines=nl) for l0, nl in parts]
    out, err = [None] * R, []
    try:
        for q, c in enumerate(ctxs):
            c.comm_init_local(g, q, max(nl for _, nl in parts))
        if transport == "xchg":
            for c in ctxs:
                c.xchg_local()
        for c in ctxs:
            c.set_precond("cheb", (8.2, 0.2), degree)

        def work(q):
            try:
                out[q] = _arnoldi_steps(ctxs[q], steps) + (ctxs[q].res_info()["cheb_sten"],)
            except Exception as e:  # pragma: no cover - reported below
                err.append(e)

        th = [threading.Thread(target=work, args=(q,)) for q in range(R)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        assert not err, err
        # the stage-0 route on every rank, or (thin slab) on none
        assert {o[3] for o in out} == ({0} if split == "thin" else {1}), [o[3] for o in out]
        for o in out:  # replicated host values: identical on every rank
            assert o[0] == out[0][0] and all(np.array_equal(a, b) for a, b in zip(o[1], out[0][1]))
        assert out[0][0] == pytest.approx(b0, rel=1e-12)
        for a, b in zip(out[0][1], H0):
            assert np.allclose(a, b, rtol=1e-11, atol=1e-13 * np.abs(b).max()), (a, b)
        v = np.concatenate([o[2] for o in out])
        assert np.allclose(v, v0, rtol=1e-10, atol=1e-12 * np.abs(v0).max())
    finally:
        for c in ctxs:
            c.close()
        g.close()
