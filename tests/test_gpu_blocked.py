"""The opt-in blocked-projection MGS-R step (GK_TUNE_RES_BLOCK = S, k_mgs_blk,
gmres_amd/csrc/gk_blk.hpp) against the reference's own runs.

The blocked step groups each sweep's projections into blocks of S columns and
closes a block with ONE in-launch all-gather (its S dots and the Gram terms of
its newest column); h follows MGS's exact-arithmetic recurrence
h_k = <w,V_k> - sum_{l<k} h_l <V_l,V_k>.  It is NOT bit-identical to the strict
MGS-R step (gmres_mgsr.f90:341-360), so it is held to the residual-history
contract of SURVEY 8c (rtol 1e-5, atol 1e-13 per restart cycle; iterations to
tol within +-1 %; ||x - 1||_inf < 1e-9) against the reference's runs
(tests/golden/reference_runs.json, the reference built from its sources), and
the measured deviation is printed (pytest -s) so the margin is on record.

Coverage: both block sizes, every instantiation of the kernel (the register,
column-cache and w-only builds, selected by the chunks per workgroup -- forced
here by sharing the device's CUs, GK_TUNE_RES_SHARE), ragged and odd-length
slabs (streamed part, tail element), and 2 / 4 row-block ranks on one GPU
through the device exchange (the in-launch rank hop carrying several values).
"""
import json
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REF = json.load(open(os.path.join(HERE, "golden", "reference_runs.json")))


def _tune(c, S, share=1):
    """S = 2 / 4: the blocked step; S = 0: the strict step on the prefetching
    blocked kernel (GK_TUNE_RES_PF)."""
    from gmres_amd import _native as nat

    if S == 0:
        c.tune(nat.GK_TUNE_RES_PF, 1)
    else:
        c.tune(nat.GK_TUNE_RES_BLOCK, S)
    if share > 1:
        c.tune(nat.GK_TUNE_RES, 1)
        c.tune(nat.GK_TUNE_RES_SHARE, share)
    c.tune(nat.GK_TUNE_RES_TIMEOUT_MS, 10000)


def _run(N, m, S, cycles, share=1, prec="identity", tol=1e-15, want_x=False):
    import gmres_amd as ga

    with ga.Context(N, m) as c:
        c.set_precond(prec, (8.2, 0.2), 8)
        c.set_rhs_ones()
        _tune(c, S, share)
        plan = c.res_info()
        c.profile(True)
        c.profile_reset()
        r = ga.gmres_mgsr(c, tol, max_cycles=cycles, want_verr=False, want_hist=True, want_x=want_x)
        return r, plan, c.profile_read()


def _dev(gpu, ref):
    g, r = np.asarray(gpu, dtype=float), np.asarray(ref, dtype=float)
    k = min(len(g), len(r))
    return float(np.max(np.abs(g[:k] - r[:k]) / np.abs(r[:k])))


def _contract(gpu, ref, rtol=1e-5, atol=1e-13):
    k = min(len(gpu), len(ref))
    assert k >= 1
    g, r = np.asarray(gpu[:k]), np.asarray(ref[:k])
    bad = np.abs(g - r) > rtol * np.abs(r) + atol
    assert not bad.any(), f"cycles {np.nonzero(bad)[0].tolist()} deviate: gpu={g} ref={r}"


@pytest.mark.parametrize("S", [2, 4])
def test_blocked_1024_twelve_cycles_vs_reference(S):
    """Config 2 (1024^2, m = 95): twelve restart cycles against the reference's
    own gmres_mgsr_omp history; every Arnoldi step one blocked resident launch."""
    g = REF["mgsr_omp_identity_1024_m95_12cyc_t8"]["hist_res"]
    r, plan, prof = _run(1024, 95, S, 12)
    assert plan["variant"] == "blocked" and plan["blk"] == S, plan
    assert prof["res"][1] >= 95 * 12 and prof["proj"][1] <= 1, prof
    assert r.n_cycles == 12
    print(f"\n[blocked S={S}] 1024^2 12 cycles: max rel dev vs reference {_dev(r.hist_res, g):.2e}")
    _contract(r.hist_res, g)


@pytest.mark.parametrize("S", [2, 4])
def test_blocked_4096_two_cycles_vs_reference(S):
    """The north-star grid (4096^2, m = 95; the w-only build): both timed cycles
    of the bench leg against the reference's own run."""
    g = REF["mgsr_omp_identity_4096_m95_2cyc_t8"]["hist_res"]
    r, plan, prof = _run(4096, 95, S, 2)
    assert plan["variant"] == "blocked" and plan["blk"] == S and plan["wt"] == 256, plan
    assert prof["res"][1] >= 95 * 2, prof
    print(f"\n[blocked S={S}] 4096^2 2 cycles: max rel dev vs reference {_dev(r.hist_res, g):.2e}")
    _contract(r.hist_res, g)


@pytest.mark.parametrize("S", [2, 4])
def test_blocked_128_converges_like_reference(S):
    """Config 1 (128^2, m = 30) to tol 1e-15: iterations within +-1 % of the
    reference's 3592, the solution within 1e-9, the history within the contract
    while it is above the chaotic floor."""
    g = REF["mgsr_omp_identity_128_m30"]
    r, plan, _ = _run(128, 30, S, 1000, want_x=True)
    assert plan["variant"] == "blocked", plan
    its = r.iterations
    print(f"\n[blocked S={S}] 128^2: {its} iterations (reference {g['iterations']})")
    assert abs(its - g["iterations"]) <= 0.01 * g["iterations"]
    assert r.final_err[r.n_out - 1] < 1e-15
    assert np.max(np.abs(r.x - 1.0)) < 1e-9
    hi = [k for k, v in enumerate(g["hist_res"]) if v > 1e-10]
    _contract(r.hist_res[: len(hi)], g["hist_res"][: len(hi)])


# share -> the instantiation a 1024^2 slab selects with 256 / share workgroups
SHARES = [(1, 4, 512), (2, 8, 512), (4, 16, 512), (8, 32, 512), (16, None, 256)]
# (S = 4 at 8 chunks of 512: the one-wave build, 16 chunks of 256 -- gk_blk.hip BlkCfg<4>)
S4_ONEWAVE = {(2, 8, 512): (16, 256)}


@pytest.mark.parametrize("S", [2, 4])
@pytest.mark.parametrize("share,chunks,wt", SHARES)
def test_blocked_every_instantiation(S, share, chunks, wt):
    """Each k_mgs_blk build (4 / 8 / 16 / 32 register chunks of w with the block
    cache, and the w-only build -- whose S = 4 geometry leaves two chunks per
    workgroup streamed) on the 1024^2 slab, three cycles against the reference."""
    g = REF["mgsr_omp_identity_1024_m95_3cyc_t8"]["hist_res"]
    r, plan, prof = _run(1024, 95, S, 3, share=share)
    if S == 4 and (share, chunks, wt) in S4_ONEWAVE:
        chunks, wt = S4_ONEWAVE[(share, chunks, wt)]
    assert plan["variant"] == "blocked" and plan["G"] == 256 // share and plan["wt"] == wt, plan
    if chunks is not None:
        assert plan["r2e"] == chunks, plan
    assert prof["res"][1] >= 95 * 3, prof
    print(f"\n[blocked S={S} share={share}] {plan}: max rel dev {_dev(r.hist_res, g):.2e}")
    _contract(r.hist_res, g)


@pytest.mark.parametrize("S", [2, 4])
@pytest.mark.parametrize("N,m", [(127, 30), (100, 20), (96, 7)])
def test_blocked_ragged_slabs_vs_oracle(oracle, S, N, m):
    """Odd n (the tail element), partial chunks (the streamed part) and small m
    (blocks shorter than S at every step): ten cycles against the oracle's
    gmres_mgsr_omp (bit-exact vs the reference's serial runs)."""
    r, plan, _ = _run(N, m, S, 10)
    assert plan["variant"] == "blocked"
    ref = oracle.gmres_mgsr(oracle.rhs_ones(N), N, m, variant=oracle.MGSR_OMP, max_cycles=10)
    print(f"\n[blocked S={S}] {N}^2 m={m}: max rel dev vs oracle {_dev(r.hist_res, ref.hist_res):.2e}")
    _contract(r.hist_res, ref.hist_res)


@pytest.mark.parametrize("S", [2, 4, 0])
@pytest.mark.parametrize("N,R", [(1448, 2), (2048, 4)])
def test_blocked_row_block_ranks(S, N, R):
    """R row-block ranks on one GPU through the device exchange, 256 / R
    workgroups each: the blocked step's multi-value all-gather and rank-total hop
    (value slot v of each replica) -- one cycle against a single-context blocked
    run (1e-9; only the dot summation order differs) and every rank taking the
    same decisions.  S = 0: the strict step on the prefetching kernel
    (GK_TUNE_RES_PF), whose split prefetch (BLK_PF_SPLIT: the non-polling waves
    prefetch so the rank-total pusher is not delayed) exists for this N-rank case."""
    import gmres_amd as ga

    single, _, _ = _run(N, 95, S, 1)
    parts = ga.slab_partition(N, R)
    g = ga.LocalGroup(R)
    ctxs = [ga.Context(N, 95, device=0, line0=l0, nlines=nl) for l0, nl in parts]
    out, err = [None] * R, []
    try:
        for r, c in enumerate(ctxs):
            c.comm_init_local(g, r, max(nl for _, nl in parts))
        for c in ctxs:
            c.xchg_local()
            _tune(c, S, share=R)
        plans = [c.res_info() for c in ctxs]
        assert all(p["variant"] == "blocked" and p["blk"] == max(S, 1) and p["G"] == 256 // R for p in plans), plans

        def work(q):
            try:
                c = ctxs[q]
                c.set_rhs_ones()
                c.profile(True)
                c.profile_reset()
                out[q] = (ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False, want_hist=True), c.profile_read())
            except Exception as e:  # pragma: no cover - reported below
                err.append(e)

        th = [threading.Thread(target=work, args=(q,)) for q in range(R)]
        for t in th:
            t.start()
        for t in th:
            t.join(100)
        assert not err, err
        assert all(o is not None for o in out)
    finally:
        for c in ctxs:
            c.close()
        g.close()
    res = [o[0] for o in out]
    assert all(np.array_equal(res[0].hist_res, x.hist_res) for x in res)
    assert all(np.array_equal(res[0].final_err, x.final_err) for x in res)
    for _, prof in out:
        assert prof["res"][1] >= 95 and prof["proj"][1] <= 1, prof
    assert res[0].hist_res[0] == pytest.approx(single.hist_res[0], rel=1e-9)
    assert np.allclose(res[0].final_err[:95], single.final_err[:95], rtol=1e-6, atol=0)


def test_step_change_inside_a_cycle_waits_for_the_next_cycle():
    """the blocked step reads Gram rows only a blocked step of the same
    cycle wrote, so GK_TUNE_RES_BLOCK / GK_TUNE_RES_PF set while a cycle is open
    apply from the next gk_mgs_cycle_start: the next solve equals a fresh blocked
    solve bit for bit."""
    import gmres_amd as ga
    from gmres_amd import _native as nat

    with ga.Context(1024, 95) as c:
        c.set_rhs_ones()
        ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)  # leaves a cycle open
        c.tune(nat.GK_TUNE_RES_BLOCK, 2)
        assert c.res_info()["blk"] == 1  # pending
        r2 = ga.gmres_mgsr(c, 1e-15, max_cycles=2, want_verr=False, want_hist=True)
        assert c.res_info()["blk"] == 2
        c.tune(nat.GK_TUNE_RES_BLOCK, 1)
        c.tune(nat.GK_TUNE_RES_PF, 1)
        assert c.res_info()["blk"] == 2
        ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)
        assert c.res_info()["blk"] == 1 and c.res_info()["variant"] == "blocked"
    fresh, _, _ = _run(1024, 95, 2, 2)
    assert np.array_equal(r2.hist_res, fresh.hist_res)
    assert np.array_equal(r2.final_err, fresh.final_err)


def test_blocked_knob_rejects_other_sizes():
    import gmres_amd as ga
    from gmres_amd import _native as nat

    with ga.Context(64, 10) as c:
        with pytest.raises(Exception):
            c.tune(nat.GK_TUNE_RES_BLOCK, 3)
        c.tune(nat.GK_TUNE_RES_BLOCK, 2)
        assert c.res_info()["blk"] == 2
        assert c.res_info(hh=True)["blk"] == 1  # the reflection chains stay strict
        with pytest.raises(Exception, match="unknown tuning key"):  # the look-ahead build (removed, round 5)
            c.tune(26, 1)



# ----------------------------------------------------- strict on the prefetch ---
# GK_TUNE_RES_PF: the STRICT MGS-R step (blocks of 1: one all-gather per projection, the
# reference's projection order) on k_mgs_blk's LDS prefetch of the next dot column.  Only
# the in-thread dot summation order differs from the strict kernels: held to the strict
# path's 1e-9 per cycle.


@pytest.mark.parametrize("share,chunks", [(1, 4), (2, 8), (4, 16), (8, 32)])
def test_strict_prefetch_build_vs_reference(share, chunks):
    from gmres_amd import _native as nat
    import gmres_amd as ga

    g = REF["mgsr_omp_identity_1024_m95_12cyc_t8"]["hist_res"]
    with ga.Context(1024, 95) as c:
        c.set_rhs_ones()
        c.tune(nat.GK_TUNE_RES_PF, 1)
        if share > 1:
            c.tune(nat.GK_TUNE_RES, 1)
            c.tune(nat.GK_TUNE_RES_SHARE, share)
        plan = c.res_info()
        c.profile(True)
        c.profile_reset()
        r = ga.gmres_mgsr(c, 1e-15, max_cycles=12, want_verr=False, want_hist=True)
        prof = c.profile_read()
    assert plan["variant"] == "blocked" and plan["blk"] == 1 and plan["r2e"] == chunks, plan
    assert prof["res"][1] >= 95 * 12 and prof["proj"][1] <= 1, prof
    print(f"\n[strict S=1 share={share}] 1024^2 12 cycles: max rel dev vs reference {_dev(r.hist_res, g):.2e}")
    assert np.allclose(r.hist_res, g, rtol=1e-9, atol=0)


def test_strict_prefetch_build_ranks_and_ragged(oracle):
    """Ragged slabs against the oracle (1e-9 over ten cycles) and the 1448^2 grid
    (the 4096^2 / 8 load, single context) against the reference's own cycle; the
    row-block ranks of this step are test_blocked_row_block_ranks[S=0]."""
    from gmres_amd import _native as nat
    import gmres_amd as ga

    for N, m in ((127, 30), (100, 20), (96, 7)):
        with ga.Context(N, m) as c:
            c.set_rhs_ones()
            c.tune(nat.GK_TUNE_RES_PF, 1)
            assert c.res_info()["blk"] == 1 and c.res_info()["variant"] == "blocked"
            r = ga.gmres_mgsr(c, 1e-15, max_cycles=10, want_verr=False, want_hist=True)
        ref = oracle.gmres_mgsr(oracle.rhs_ones(N), N, m, variant=oracle.MGSR_OMP, max_cycles=10)
        k = min(len(r.hist_res), len(ref.hist_res))
        hi = [i for i in range(k) if ref.hist_res[i] > 1e-10]
        assert np.allclose(np.asarray(r.hist_res)[hi], np.asarray(ref.hist_res)[hi], rtol=1e-9, atol=0), (N, m)
    g = REF["mgsr_omp_identity_1448_m95_1cyc_t8"]["hist_res"]
    with ga.Context(1448, 95) as c:
        c.set_rhs_ones()
        c.tune(nat.GK_TUNE_RES_PF, 1)
        assert c.res_info()["r2e"] == 8
        r = ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False, want_hist=True)
    assert r.hist_res[0] == pytest.approx(g[0], rel=1e-9)
