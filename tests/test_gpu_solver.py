"""End-to-end GMRES(m) parity on the GPU (Fortran host + HIP kernels) against
the CPU oracle and the reference's own recorded outputs (tests/golden).

Tolerance contract (derived from the reference vs itself at 1 vs 8 OpenMP
threads): per-cycle true residual within rtol 1e-5 / atol 1e-13 on
the common cycle prefix, iterations to tol within +-1 %, ||x-1||_inf < 1e-9.
"""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "reference_known_answers.json")))


def _hist_close(gpu, ref, rtol=1e-5, atol=1e-13):
    k = min(len(gpu), len(ref))
    assert k >= 1
    dev = np.abs(np.asarray(gpu[:k]) - np.asarray(ref[:k]))
    bad = dev > rtol * np.abs(ref[:k]) + atol
    assert not bad.any(), f"cycles {np.nonzero(bad)[0].tolist()} deviate: gpu={gpu[:k]} ref={ref[:k]}"


def _hist_close_hh(gpu, ref):
    """Householder tolerance, derived from the reference restatement against
    itself at 1 vs 8 OpenMP threads (128^2, m=30): 1e-12 relative while
    r > 1e-6, then up to 1.1e-4 relative (cycles 45-80) and 8e-3 at the 1e-15
    floor.  Tiers: r > 1e-6 -> rtol 1e-8; r > 1e-12 -> rtol 1e-3; below -> 5e-2."""
    k = min(len(gpu), len(ref))
    g, r = np.asarray(gpu[:k]), np.asarray(ref[:k])
    rtol = np.where(r > 1e-6, 1e-8, np.where(r > 1e-12, 1e-3, 5e-2))
    bad = np.abs(g - r) > rtol * r + 1e-16
    assert not bad.any(), f"cycles {np.nonzero(bad)[0].tolist()} deviate"


def _solve(N, m, prec="identity", method="mgsr", variant=1, max_cycles=1000, degree=8, want_hist=True):
    import gmres_amd as ga

    with ga.Context(N, m) as ctx:
        ctx.set_precond(prec, (8.2, 0.2), degree)
        ctx.set_rhs_ones()
        if method == "mgsr":
            return ga.gmres_mgsr(ctx, 1e-15, variant=variant, max_cycles=max_cycles, want_hist=want_hist)
        if method == "hh":  # gmres_hh_omp
            return ga.gmres_hh(ctx, 1e-15, precondition=False, max_cycles=max_cycles, want_hist=want_hist)
        return ga.gmres_hh(ctx, 1e-15, precondition=True, max_cycles=max_cycles, want_hist=want_hist)


def test_mgsr_128_identity_matches_reference(oracle):
    """Config 1: 128^2, m=30, no preconditioner, to tol 1e-15."""
    g = GOLD["mgsr_identity_128_m30"]
    r = _solve(128, 30, "identity")
    assert abs(r.iterations - g["iterations"]) <= 0.01 * g["iterations"]
    assert r.final_err[r.n_out - 1] < 1e-15
    assert np.max(np.abs(r.x - 1.0)) < 1e-9
    ref = oracle.gmres_mgsr(oracle.rhs_ones(128), 128, 30, variant=oracle.MGSR_OMP)
    _hist_close(r.hist_res, ref.hist_res)
    # the last cycle differs between runs that end a few iterations apart (3592 vs
    # 3587-3589 in the reference itself): its final_err is compared at a fixed
    # cycle count below (test_mgsr_128_final_err_fixed_cycles)


def test_mgsr_128_final_err_fixed_cycles(oracle):
    """final_err(1:m) step by step and the per-cycle residuals after exactly 3
    cycles (config 1): the oracle against itself at 1 vs 2/4/8 OpenMP threads
    differs by <= 1.5e-14 relative in final_err and 8.6e-15 in the residuals;
    the tree-reduced device dots get 1e-10."""
    r = _solve(128, 30, "identity", max_cycles=3)
    ref = oracle.gmres_mgsr(oracle.rhs_ones(128), 128, 30, variant=oracle.MGSR_OMP, max_cycles=3)
    assert r.n_out == ref.n_out == 30 and r.n_cycles == 3 and len(r.hist_res) == len(ref.hist_res)
    assert np.allclose(r.final_err[:30], ref.final_err[:30], rtol=1e-10, atol=0)
    assert np.allclose(r.hist_res, ref.hist_res, rtol=1e-10, atol=0)


def test_mgsr_128_mf_variant(oracle):
    r = _solve(128, 30, "identity", variant=0)
    ref = oracle.gmres_mgsr(oracle.rhs_ones(128), 128, 30, variant=oracle.MGSR_MF)
    assert abs(r.iterations - ref.iterations) <= 0.01 * ref.iterations
    _hist_close(r.hist_res, ref.hist_res)


def test_mgsr_128_cbpr2_matches_reference(oracle):
    g = GOLD["mgsr_cbpr2_128_m30"]
    r = _solve(128, 30, "cbpr2")
    assert abs(r.iterations - g["iterations"]) <= 0.01 * g["iterations"]
    assert np.max(np.abs(r.x - 1.0)) < 1e-9
    ref = oracle.gmres_mgsr(oracle.rhs_ones(128), 128, 30, prec=oracle.PREC_CBPR2, variant=oracle.MGSR_OMP)
    _hist_close(r.hist_res, ref.hist_res)


def test_mgsr_cheb8(oracle):
    """Chebyshev(8) (build-defined extension of config 3) vs the oracle."""
    r = _solve(128, 30, "cheb", degree=8)
    ref = oracle.gmres_mgsr(oracle.rhs_ones(128), 128, 30, prec=oracle.PREC_CHEB, degree=8,
                            variant=oracle.MGSR_OMP)
    assert abs(r.iterations - ref.iterations) <= max(1, 0.01 * ref.iterations)
    _hist_close(r.hist_res, ref.hist_res)
    assert np.max(np.abs(r.x - 1.0)) < 1e-9


def test_hh_128_identity_matches_reference(oracle):
    g = GOLD["hh_identity_128_m30"]
    r = _solve(128, 30, method="hh")
    assert r.iterations == g["iterations"]  # gmres_hh_omp always runs full cycles
    ref = oracle.gmres_hh(oracle.rhs_ones(128), 128, 30, midcycle_exit=0)
    _hist_close_hh(r.hist_res, ref.hist_res)
    assert r.v_err[r.n_out - 1] < 1e-25  # squared metric, reference ~1e-30


def test_hh_128_cbpr2_matches_reference(oracle):
    g = GOLD["hh_cbpr2_128_m30"]
    r = _solve(128, 30, "cbpr2", method="hh_prec")
    assert abs(r.iterations - g["iterations"]) <= 0.01 * g["iterations"]
    ref = oracle.gmres_hh(oracle.rhs_ones(128), 128, 30, prec=oracle.PREC_CBPR2, midcycle_exit=1)
    _hist_close_hh(r.hist_res, ref.hist_res)


@pytest.mark.parametrize("prec,key", [("identity", "mgsr_identity_1024_m95"), ("cbpr2", "mgsr_cbpr2_1024_m95")])
def test_1024_three_cycles_vs_reference(prec, key):
    """Config 2 size: the reference's own per-cycle true residuals (serial run)."""
    g = GOLD[key]
    r = _solve(1024, 95, prec, max_cycles=3)
    _hist_close(r.hist_res, g["cycle_true_residual"], rtol=1e-9, atol=0.0)


def test_1024_hh_three_cycles_vs_reference():
    g = GOLD["hh_identity_1024_m95"]
    r = _solve(1024, 95, method="hh", max_cycles=3)
    _hist_close(r.hist_res, g["cycle_true_residual"], rtol=1e-9, atol=0.0)


REF_RUNS = json.load(open(os.path.join(HERE, "golden", "reference_runs.json")))


def _history_pinned(gpu, ref, rtol=1e-9, floor=1e-6):
    """EVERY cycle of the reference's history within rtol while its residual is
    above `floor` (the reference at 1 vs 8 threads agrees to 1.5e-13
    there; below ~1e-6 the history is chaotic and the 1e-5 contract applies)."""
    assert len(gpu) >= len(ref), (len(gpu), len(ref))
    g, r = np.asarray(gpu[: len(ref)]), np.asarray(ref)
    tol = np.where(r > floor, rtol, 1e-5)
    dev = np.abs(g - r) / r
    assert (dev <= tol).all(), f"cycles {np.nonzero(dev > tol)[0].tolist()} deviate: {dev.tolist()}"


@pytest.mark.parametrize("method,prec,key", [
    ("mgsr", "identity", "mgsr_omp_identity_1024_m95_12cyc_t8"),
    ("mgsr", "cbpr2", "mgsr_omp_cbpr2_1024_m95_12cyc_t8"),
    ("hh", "identity", "hh_omp_identity_1024_m95_12cyc_t8"),
])
def test_1024_twelve_cycle_history_vs_reference(method, prec, key):
    """Config 2 size, twelve restart cycles: the whole per-cycle true-residual
    history of the reference's own gmres_mgsr_omp / gmres_hh_omp run (oracle/_ref,
    8 threads; tests/golden/make_ref_fixtures.py) -- gmres_mgsr.f90:309-413,
    gmres_hh.f90:420-563 -- cycle by cycle at 1e-9."""
    g = REF_RUNS[key]
    assert len(g["hist_res"]) == 12
    r = _solve(1024, 95, prec, method=method, max_cycles=12)
    assert r.n_cycles == 12
    _history_pinned(r.hist_res, g["hist_res"])


# v_err by value (a9, a12, f1).  Both diagnostics measure rounding noise, and
# the reference's own figure is dominated by the rounding of the sequential
# dot_product that MEASURES it (one n-term running sum per dot), not by the
# basis: a tree-reduced Gram of the same basis gives ~10x (MGS-R) / ~1000x
# (HH) smaller values (measured on this device).  So the device evaluates the
# diagnostics in the reference's order (GK_TUNE_VERR_ORDER, default), and
# parity is pinned in two parts:
#  (a) BIT-EXACT: the device-reported v_err equals the reference's formula,
#      with the reference's dot_product (oracle.dot, 1 thread), evaluated on
#      the host on the basis copied off the device (Householder: rebuilt from
#      the device reflectors, and the device's rebuilt basis equals that);
#  (b) STATISTICAL: that value against the oracle's v_err of its own run,
#      within the oracle's own 1-vs-N-thread spread (the bases differ by
#      reduction order only).  Spread of the oracle against itself at 1 vs
#      2/4/8 OpenMP threads (64^2 m=20 2 cycles, 128^2 m=30 3 cycles and to
#      convergence):
#        MGS-R v_err(2:n_out+1): last (cumulative) entry within 0.24 decades,
#              entrywise median <= 0.27, entrywise max 0.54 decades; over every
#              pair of 1..8 threads, two runs (tools/verr_spread.py,
#              profiles/r05/verr_oracle_spread_r05.txt; the threaded oracle is
#              not run-to-run deterministic): last 0.31, median 0.36, entrywise
#              max 1.25 decades -- the first entries, a few rounding errors each;
#        HH calculate_verr(2:n_out): sum within 0.36 decades, entrywise median
#              <= 0.65, entrywise max 2.8 decades (single terms are pure noise).
#      Tolerances: about twice the measured spread, in decades.
def _decades(a, b):
    return np.abs(np.log10(np.asarray(a, dtype=np.float64) / np.asarray(b, dtype=np.float64)))


def _mgs_verr_close(a, b):
    d = _decades(a, b)
    assert d[-1] <= 0.6, (a[-1], b[-1])
    assert np.median(d) <= 0.7 and d.max() <= 2.5, d


def _hh_verr_close(a, b, below=0.7, above=0.7):
    """Sum within [-below, +above] decades of the oracle's; entrywise, the
    median |decades| within 0.8 (two-sided band) or the median signed ratio
    within [-below, +0.8] (one-sided band, below > 0.7)."""
    a, b = np.asarray(a), np.asarray(b)
    assert np.all(a > 0) and np.all(a < 1e-27)
    r = np.log10(a.sum() / b.sum())
    assert -below <= r <= above, (a.sum(), b.sum())
    if below <= 0.7:
        assert np.median(_decades(a, b)) <= 0.8, _decades(a, b)
    else:
        assert -below <= np.median(np.log10(a / b)) <= 0.8, np.log10(a / b)


def _solve_keep(N, m, prec, method, cycles):
    """Solve, then copy the device bases out before the context closes."""
    import gmres_amd as ga

    with ga.Context(N, m) as ctx:
        ctx.set_precond(prec, (8.2, 0.2), 8)
        ctx.set_rhs_ones()
        if method == "mgsr":
            r = ga.gmres_mgsr(ctx, 1e-15, max_cycles=cycles)
            return r, [ctx.get_basis(k, 0) for k in range(r.n_out + 1)], None
        r = ga.gmres_hh(ctx, 1e-15, precondition=method == "hh_prec", max_cycles=cycles)
        return r, [ctx.get_basis(k, 0) for k in range(r.n_out)], [ctx.get_basis(k, 1) for k in range(r.n_out)]


@pytest.mark.parametrize("N,m,cycles", [(64, 20, 2), (128, 30, 3)])
def test_mgsr_verr_by_value(oracle, N, m, cycles):
    """a9: the MGS-R orthogonality diagnostic (gmres_mgsr.f90:414-420)."""
    from tests import verr_host as vh

    r, V, _ = _solve_keep(N, m, "identity", "mgsr", cycles)
    ref = oracle.gmres_mgsr(oracle.rhs_ones(N), N, m, variant=oracle.MGSR_OMP, max_cycles=cycles)
    assert r.n_out == ref.n_out == m
    host = vh.mgs_verr(V, m, vh.ref_dot(oracle))
    assert np.array_equal(r.v_err[:m + 1], host[:m + 1])                   # (a)
    _mgs_verr_close(r.v_err[1:m + 1], ref.v_err[1:m + 1])                  # (b)


@pytest.mark.parametrize("N,m,cycles", [(64, 20, 2), (128, 30, 3)])
@pytest.mark.parametrize("method", ["hh", "hh_prec"])
def test_hh_verr_by_value(oracle, N, m, cycles, method):
    """a12 / f1: calculate_verr (gmres_hh.f90:568-593) for gmres_hh_omp and
    gmres_hh_prec_omp."""
    from tests import verr_host as vh

    prec = "identity" if method == "hh" else "cbpr2"
    r, P, Vb = _solve_keep(N, m, prec, method, cycles)
    ref = oracle.gmres_hh(oracle.rhs_ones(N), N, m, prec=oracle.PREC_NAMES[prec],
                          midcycle_exit=int(method == "hh_prec"), max_cycles=cycles)
    n = r.n_out
    assert n == ref.n_out == m
    dot = vh.ref_dot(oracle)
    Vh = vh.hh_rebuild(P, n, dot)
    assert all(np.array_equal(a, b) for a, b in zip(Vb, Vh))               # (a) the rebuilt basis
    assert np.array_equal(r.v_err[1:n], vh.hh_verr_of_basis(Vh, n, dot)[1:n])  # (a) the diagnostic
    _hh_verr_close(r.v_err[1:n], ref.v_err[1:n])                           # (b)


def test_hh_verr_vs_reference_run(oracle):
    """The reference's own 128^2 m=30 gmres_hh_omp run to convergence
    (tests/golden/reference_runs.json; README's "~1e-30", last entry 9.5e-31).
    After 120 cycles the device basis is MORE orthogonal than the reference's:
    measured 1.08 decades below it (the reflectors are normalised by
    tree-reduced norms, closer to unit length than the reference's running
    sums make them), so the band is one-sided: never above the reference by
    more than the thread spread, at most 1.5 decades below."""
    from tests import verr_host as vh

    ref = json.load(open(os.path.join(HERE, "golden", "reference_runs.json")))["hh_omp_identity_128_m30"]
    r, P, _ = _solve_keep(128, 30, "identity", "hh", 1000)
    assert r.n_out == ref["n_out"] == 30 and r.iterations == ref["iterations"]
    assert np.array_equal(r.v_err[1:30], vh.hh_verr(P, 30, vh.ref_dot(oracle))[1:30])
    _hh_verr_close(r.v_err[1:30], ref["v_err"][1:30], below=1.5)


def test_hh_verr_two_sided_with_reference_order_norms(oracle):
    """with the reflector norms taken in the reference's own
    order (GK_TUNE_HH_NORM_ORDER: flang-rt's NORM2 running max + scaled sum,
    gmres_hh.f90:251-253,307,315) the device basis carries the reference's
    normalisation rounding, and its calculate_verr after the 128^2 m=30 run to
    convergence falls inside the TWO-sided band of the reference's own figure
    (the default tree-reduced norms sit 1.08 decades below it:
    test_hh_verr_vs_reference_run).  (a) by value as always: the device figure
    equals the reference's formula on the device basis."""
    import gmres_amd as ga
    from gmres_amd import _native as nat
    from tests import verr_host as vh

    ref = json.load(open(os.path.join(HERE, "golden", "reference_runs.json")))["hh_omp_identity_128_m30"]
    with ga.Context(128, 30) as ctx:
        ctx.tune(nat.GK_TUNE_HH_NORM_ORDER, 1)
        ctx.set_rhs_ones()
        r = ga.gmres_hh(ctx, 1e-15, precondition=False, max_cycles=1000)
        P = [ctx.get_basis(k, 0) for k in range(r.n_out)]
    assert r.n_out == ref["n_out"] == 30 and abs(r.iterations - ref["iterations"]) <= 0.01 * ref["iterations"]
    assert np.array_equal(r.v_err[1:30], vh.hh_verr(P, 30, vh.ref_dot(oracle))[1:30])
    d = np.log10(np.sum(r.v_err[1:30]) / np.sum(ref["v_err"][1:30]))
    print(f"\n[hh norm order] v_err sum vs reference: {d:+.2f} decades; median entry "
          f"{np.median(np.log10(np.asarray(r.v_err[1:30]) / np.asarray(ref['v_err'][1:30]))):+.2f}")
    _hh_verr_close(r.v_err[1:30], ref["v_err"][1:30])  # two-sided: +-0.7 decades, median |d| <= 0.8


def test_true_residual_and_solution(oracle):
    import gmres_amd as ga

    N = 96
    with ga.Context(N, 25) as ctx:
        ctx.set_rhs_ones()
        b = ctx.apply(np.ones(N * N), 0)
        assert np.array_equal(b, oracle.rhs_ones(N))
        r = ga.gmres_mgsr(ctx, 1e-15, want_hist=True)
        assert ctx.true_residual() == pytest.approx(r.hist_res[-1], rel=1e-12)


@pytest.mark.parametrize("method", ["mgsr", "hh"])
def test_solution_kept_in_hbm(method):
    """want_x = False (the bench's timed solve): the host x is not written and
    the device x read afterwards is the one a downloading solve returns."""
    import gmres_amd as ga

    N, m = 64, 12
    out = []
    for want_x in (True, False):
        with ga.Context(N, m) as ctx:
            ctx.set_rhs_ones()
            if method == "mgsr":
                r = ga.gmres_mgsr(ctx, 1e-15, max_cycles=3, want_verr=False, want_x=want_x)
            else:
                r = ga.gmres_hh(ctx, 1e-15, max_cycles=3, want_verr=False, want_x=want_x)
            assert r.x.size == (N * N if want_x else 0)
            out.append((r.x if want_x else ctx.get_x(), r.n_cycles, r.n_out))
    assert out[0][1:] == out[1][1:]
    assert np.array_equal(out[0][0], out[1][0])


@pytest.mark.slow
@pytest.mark.parametrize("prec,key", [("identity", "mgsr_identity_4096_m95"), ("cbpr2", "mgsr_cbpr2_4096_m95")])
def test_4096_first_cycle_vs_reference(prec, key):
    """North-star size (4096^2, m=95): cycle-1 true residual vs the reference
    run recorded in the survey (4 significant digits published)."""
    g = GOLD[key]
    r = _solve(4096, 95, prec, max_cycles=1, want_hist=True)
    assert r.hist_res[0] == pytest.approx(g["cycle_true_residual"][0], rel=6e-5)


def test_fortran_driver_runs():
    """The Fortran drop-in driver (tests/test_poisson_mf.f90 CLI) on the GPU."""
    exe = os.path.join(os.path.dirname(HERE), "gmres_amd", "lib", "test_mfp_hip")
    out = subprocess.run([exe, "128", "30"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = [l for l in out.stdout.splitlines() if "Iterations until convergence" in l]
    assert len(lines) == 2
    its = [int(l.split(":")[1].split()[0]) for l in lines]
    for it in its:  # HH+cbpr2 and MGSR+cbpr2: 1056 in the reference
        assert abs(it - 1056) <= 11, out.stdout


@pytest.mark.parametrize("N,k", [(16, 60), (32, 80)])
def test_lanczos_bounds_match_poisson_spectrum(N, k):
    """Extreme eigenvalues of the 5-point Dirichlet Laplacian are known in closed
    form: 8 sin^2(pi / (2(N+1))) and 8 cos^2(pi / (2(N+1)))."""
    import gmres_amd as ga

    with ga.Context(N, 10) as ctx:
        lo, hi = ctx.lanczos_bounds(k)
    t = np.pi / (2 * (N + 1))
    # the low end of the spectrum converges more slowly without reorthogonalisation
    assert lo == pytest.approx(8 * np.sin(t) ** 2, rel=1e-4)
    assert hi == pytest.approx(8 * np.cos(t) ** 2, rel=1e-9)


def test_chebyshev_with_lanczos_interval_converges():
    import gmres_amd as ga

    N = 64
    with ga.Context(N, 20) as ctx:
        lo, hi = ctx.lanczos_bounds(40)
        ctx.set_precond("cheb", (hi * 1.01, lo), 6)
        ctx.set_rhs_ones()
        r = ga.gmres_mgsr(ctx, 1e-15, want_hist=True)
    assert r.final_err[r.n_out - 1] < 1e-15
    assert np.max(np.abs(r.x - 1.0)) < 1e-9


@pytest.mark.parametrize("solver,prec", [("pcg", "identity"), ("pcg", "cbpr2"), ("pbicgstab", "identity"),
                                         ("pbicgstab", "cbpr2")])
def test_short_recurrence_solvers_vs_reference_run(solver, prec):
    """pcg_omp / pbicgstab_omp against the reference's own runs (48^2, tol 1e-9,
    tests/golden/reference_runs.json): iteration count (PCG +-2, BiCGSTAB +-15 %,
    its recurrence amplifies reduction-order differences) and convergence."""
    import gmres_amd as ga

    g = json.load(open(os.path.join(HERE, "golden", "reference_runs.json")))[f"{solver}_omp_{prec}_48"]
    with ga.Context(48, 8) as ctx:
        ctx.set_precond(prec, (8.2, 0.2), 4)
        ctx.set_rhs_ones()
        x, it, res, _ = getattr(ga, solver)(ctx, 1e-9, g["m"], want_hist=True)
    assert res < 1e-9 and g["res"] < 1e-9
    assert abs(it - g["iterations"]) <= (2 if solver == "pcg" else max(3, 0.15 * g["iterations"])), (it, g["iterations"])
    assert np.max(np.abs(x - 1.0)) < 1e-6


from tests.sr_band import BAND_F, bicgstab_band  # noqa: E402


@pytest.mark.parametrize("N", [128, 256])
@pytest.mark.parametrize("solver,prec", [("pcg", "identity"), ("pcg", "cbpr2"), ("pbicgstab", "identity"),
                                         ("pbicgstab", "cbpr2")])
def test_short_recurrence_history_vs_reference(solver, prec, N):
    """pcg_omp / pbicgstab_omp (src/cg.f90:154-234, src/bicgstab.f90:91-182)
    against the reference's OWN per-iteration residual history at 128^2 and
    256^2 (tests/golden/reference_runs.json "*_hist": the reference truncated
    at every iteration k, make_ref_fixtures.py; the restatement reproduces it
    bit for bit, tests/test_reference.py).  The device's dots differ from the
    reference's running sums only in summation order.  PCG: 1e-8 relative
    while the residual is above 1e-4, 5e-2 below (the reference against itself
    at 1 vs 8 threads: <= 1.3e-12 until the last iterations); BiCGSTAB: every
    iteration inside the band the reference's own 1-vs-8-thread spread sets
    (bicgstab_band), and the iteration count within 15 %."""
    import gmres_amd as ga

    g = REF_RUNS[f"{solver}_omp_{prec}_{N}_hist"]
    it_ref, h_ref = g["iterations"], np.asarray(g["hist_res"])
    with ga.Context(N, 8) as ctx:
        ctx.set_precond(prec, (8.2, 0.2), 4)
        ctx.set_rhs_ones()
        x, it, res, hist = getattr(ga, solver)(ctx, 1e-9, 5000, want_hist=True)
    assert res < 1e-9
    k = min(len(hist), len(h_ref))
    h, r = np.asarray(hist[:k]), h_ref[:k]
    if solver == "pcg":
        assert abs(it - it_ref) <= max(2, 0.01 * it_ref), (it, it_ref)
        rt = np.where(r > 1e-4, 1e-8, 5e-2)
        dev = np.abs(h - r) / r
        print(f"\n[{solver} {prec} {N}^2] {it} vs {it_ref} iterations; max rel dev above 1e-4: "
              f"{dev[r > 1e-4].max():.2e}")
        assert np.all(dev <= rt), np.nonzero(dev > rt)[0][:10]
    else:
        assert abs(it - it_ref) <= max(3, 0.15 * it_ref), (it, it_ref)
        ok, worst = bicgstab_band(h, r, np.asarray(REF_RUNS[f"{solver}_omp_{prec}_{N}_hist_t8"]["hist_res"]))
        print(f"\n[{solver} {prec} {N}^2] {it} vs {it_ref} iterations; whole history inside the band, worst "
              f"|ln(h/r)| / ln(1 + {BAND_F:.0f} S) = {worst:.2f}")
        assert ok, worst
    assert np.max(np.abs(x - 1.0)) < 1e-6


@pytest.mark.parametrize("solver", ["pcg", "pbicgstab"])
@pytest.mark.parametrize("prec", ["identity", "cbpr2", "cheb"])
def test_short_recurrence_solvers_vs_oracle(oracle, solver, prec):
    """pcg_omp / pbicgstab_omp on the same device kernels,
    against the oracle restatement -- which reproduces the reference's own runs
    bit for bit (tests/test_reference.py); Chebyshev(k) is build-defined."""
    import gmres_amd as ga

    N, tol = 64, 1e-9
    kid = {"identity": oracle.PREC_IDENTITY, "cbpr2": oracle.PREC_CBPR2, "cheb": oracle.PREC_CHEB}[prec]
    ref_x, ref_it, ref_res, ref_hist = getattr(oracle, solver)(oracle.rhs_ones(N), N, tol, 2000, kid, degree=4)
    with ga.Context(N, 8) as ctx:
        ctx.set_precond(prec, (8.2, 0.2), 4)
        ctx.set_rhs_ones()
        x, it, res, hist = getattr(ga, solver)(ctx, tol, 2000, want_hist=True)
    assert res < tol
    k = min(len(hist), len(ref_hist))
    h, r = hist[:k], ref_hist[:k]
    if solver == "pcg":
        assert abs(it - ref_it) <= max(2, 0.03 * ref_it)
        rt = np.where(r > 1e-4, 1e-8, 5e-2)
        assert np.all(np.abs(h - r) <= rt * r), (h[:5], r[:5])
    else:
        # BiCGSTAB amplifies reduction-order differences (measured: 3e-7
        # relative by r ~ 5e-3, 1e-1 near 1e-4): compare the first decade
        # tightly, then convergence and the iteration count.
        assert abs(it - ref_it) <= max(3, 0.15 * ref_it)
        early = r > 1e-1 * r[0]
        assert np.all(np.abs(h[early] - r[early]) <= 1e-9 * r[early])
    assert np.max(np.abs(x - 1.0)) < 1e-6


def test_sweep_driver_table():
    """Fortran sweep driver prints the reference's utils.f90 table layout."""
    exe = os.path.join(os.path.dirname(HERE), "gmres_amd", "lib", "sweep_hip")
    out = subprocess.run([exe, "prec", "64", "20"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    rows = [l for l in out.stdout.splitlines() if l[:3].strip().isdigit()]
    assert len(rows) == 3
    for r in rows:
        f = r.split()
        # columns: #, Vars, Iters, Restarts, gmres(n), Tol., L2, L_inf, Residual, ||I-V.t*V||, Time, Info
        assert int(f[1]) == 64 * 64 and float(f[8]) < 1e-15 and float(f[7]) < 1e-9
