"""The CPU oracle against the reference's own recorded outputs (tests/golden/
reference_known_answers.json) and against the committed
oracle fixtures.  CPU only."""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "reference_known_answers.json")))


def test_mgsr_128_identity_bit_exact(oracle):
    """gmres_mgsr_mf on 128^2, m=30: the serial reference's iteration count
    and final_err reproduced to the last bit."""
    g = GOLD["mgsr_identity_128_m30"]
    b = oracle.rhs_ones(128)
    r = oracle.gmres_mgsr(b, 128, 30, variant=oracle.MGSR_MF)
    assert r.iterations == g["iterations"]
    assert r.cycles_out == g["cycles"]
    assert r.final_err[r.n_out - 1] == g["final_err"]
    assert r.hist_res[-1] == pytest.approx(g["true_rel_residual"], rel=1e-4)
    assert np.linalg.norm(r.x - 1.0) == pytest.approx(g["x_minus_1_l2"], rel=1e-3)
    # gmres_mgsr_omp at 1 thread is bit-identical to _mf
    r2 = oracle.gmres_mgsr(b, 128, 30, variant=oracle.MGSR_OMP)
    assert r2.iterations == g["iterations"] and r2.final_err[r2.n_out - 1] == g["final_err"]


@pytest.mark.parametrize("key,solver", [("mgsr_cbpr2_128_m30", "mgsr"), ("hh_cbpr2_128_m30", "hh_prec"),
                                        ("hh_identity_128_m30", "hh")])
def test_128_iteration_counts(oracle, key, solver):
    g = GOLD[key]
    b = oracle.rhs_ones(128)
    if solver == "mgsr":
        r = oracle.gmres_mgsr(b, 128, 30, prec=oracle.PREC_CBPR2, variant=oracle.MGSR_OMP)
    elif solver == "hh_prec":
        r = oracle.gmres_hh(b, 128, 30, prec=oracle.PREC_CBPR2, midcycle_exit=1)
    else:
        r = oracle.gmres_hh(b, 128, 30, midcycle_exit=0)
        assert r.v_err[r.n_out - 1] == pytest.approx(g["v_err_approx"], rel=0.05)
    assert r.iterations == g["iterations"]
    assert r.cycles_out == g["cycles"]


def test_1024_first_cycle_matches_reference(oracle):
    """Config 2 size, cycle 1 true residual; OpenMP 8 threads (reduction order
    differs from the serial reference only at the 1e-13 level here)."""
    b = oracle.rhs_ones(1024)
    r = oracle.gmres_mgsr(b, 1024, 95, variant=oracle.MGSR_OMP, max_cycles=1, threads=8)
    g = GOLD["mgsr_identity_1024_m95"]["cycle_true_residual"][0]
    assert r.hist_res[0] == pytest.approx(g, rel=1e-11)


def test_operators_match_fixtures(oracle):
    fx = np.load(os.path.join(HERE, "golden", "oracle_operators.npz"))
    for N in (8, 33, 64):
        x = fx[f"stvec_x_{N}"]
        assert np.array_equal(oracle.stvec(x, N), fx[f"stvec_y_{N}"])
        assert np.array_equal(oracle.precond(oracle.PREC_CBPR2, x, N), fx[f"cbpr2_z_{N}"])
        assert np.array_equal(oracle.precond(oracle.PREC_CHEB, x, N, degree=8), fx[f"cheb8_z_{N}"])


def test_stvec_matches_dense_poisson(oracle):
    """stvec equals the dense 5-point matrix of poisson.f90:13-30 applied to x."""
    N = 9
    n = N * N
    A = np.zeros((n, n))
    for j in range(N):
        for i in range(N):
            row = i + j * N
            A[row, row] = 4.0
            if i > 0:
                A[row, row - 1] = -1.0
            if i < N - 1:
                A[row, row + 1] = -1.0
            if j > 0:
                A[row, row - N] = -1.0
            if j < N - 1:
                A[row, row + N] = -1.0
    x = np.random.default_rng(0).standard_normal(n)
    assert np.allclose(oracle.stvec(x, N), A @ x, rtol=0, atol=1e-13)
    b = oracle.rhs_ones(N)
    # b = A*1 is nonzero only on the boundary: 1 on edges, 2 on corners
    assert oracle.norm2(b) == pytest.approx(np.sqrt(4 * (N - 2) + 16))


def test_cbpr2_is_degree_one_polynomial(oracle):
    """cbpr2 = (1/d + alpha) r - (alpha/d) A r with the drivers' params."""
    d, alpha = oracle.cbpr2_coeffs((8.2, 0.2))
    assert d == pytest.approx(4.2)
    assert alpha == pytest.approx(0.2516835977628125, rel=1e-15)
    N = 16
    r = np.random.default_rng(1).standard_normal(N * N)
    z = oracle.precond(oracle.PREC_CBPR2, r, N)
    assert np.allclose(z, (1 / d + alpha) * r - (alpha / d) * oracle.stvec(r, N), atol=1e-14)


def test_chebyshev_polynomial_reduces_error(oracle):
    """Chebyshev(k) approximates A^-1 on its interval: the error of z = p(A) r
    against A^-1 r shrinks with the degree for a smooth-free (high-frequency) r."""
    N = 16
    rng = np.random.default_rng(3)
    r = rng.standard_normal(N * N)
    errs = []
    for k in (1, 4, 8, 16):
        z = oracle.precond(oracle.PREC_CHEB, r, N, params=(8.0, 0.05), degree=k)
        errs.append(np.linalg.norm(r - oracle.stvec(z, N)))
    assert errs[0] > errs[1] > errs[2] > errs[3]


def test_small_solves_match_fixtures(oracle):
    fx = np.load(os.path.join(HERE, "golden", "oracle_solves.npz"))
    for N, m in ((32, 10), (32, 30)):
        b = oracle.rhs_ones(N)
        r = oracle.gmres_mgsr(b, N, m, variant=oracle.MGSR_OMP)
        key = f"mgsr_id_{N}_m{m}"
        assert np.array_equal(r.x, fx[key + "_x"])
        assert r.iterations == int(fx[key + "_iters"][0])
        r = oracle.gmres_hh(b, N, m, prec=oracle.PREC_CBPR2, midcycle_exit=1)
        key = f"hh_cbpr2_{N}_m{m}"
        assert np.array_equal(r.hist_res, fx[key + "_hist_res"])


def test_step_limit_sample(oracle):
    """The bounded CPU-baseline sample stops after step_limit Arnoldi steps."""
    b = oracle.rhs_ones(64)
    r = oracle.gmres_mgsr(b, 64, 30, variant=oracle.MGSR_OMP, step_limit=7)
    assert r.cut and np.all(np.diff(r.step_times) >= 0) and r.step_times[6] > 0


@pytest.mark.parametrize("solver", ["pcg", "pbicgstab"])
def test_short_recurrence_oracle_converges(oracle, solver):
    N = 48
    for kind in (oracle.PREC_IDENTITY, oracle.PREC_CBPR2):
        x, it, res, hist = getattr(oracle, solver)(oracle.rhs_ones(N), N, 1e-9, 5000, kind)
        assert res < 1e-9 and it == len(hist)
        assert np.max(np.abs(x - 1.0)) < 1e-6
    # the preconditioner cuts the iteration count
    _, it_id, _, _ = getattr(oracle, solver)(oracle.rhs_ones(N), N, 1e-9, 5000, oracle.PREC_IDENTITY)
    _, it_pc, _, _ = getattr(oracle, solver)(oracle.rhs_ones(N), N, 1e-9, 5000, oracle.PREC_CBPR2)
    assert it_pc < it_id
