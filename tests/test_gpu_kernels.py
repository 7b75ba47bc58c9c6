"""Kernel-level parity on the GPU: each HIP kernel against the CPU oracle
(which restates the reference Fortran in the same operation order).

Elementwise / stencil work is bit-exact (same association order, no FMA
contraction on either side); reductions differ only in summation order and
are checked to a relative 1e-13 of sum |a_i b_i|.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


@pytest.mark.parametrize("N", [2, 3, 7, 64, 127, 128, 513, 1024])
def test_poisson5_bitexact(oracle, N):
    import gmres_amd.solver as S

    rng = np.random.default_rng(N)
    x = rng.standard_normal(N * N)
    xd = _dev(x)
    yd = torch.empty_like(xd)
    S.poisson5(xd, yd, N)
    torch.cuda.synchronize()
    y = yd.cpu().numpy()
    assert np.array_equal(y, oracle.stvec(x, N))


@pytest.mark.parametrize("N,nranks", [(64, 2), (65, 3), (256, 4), (130, 7)])
def test_poisson5_slabs_with_halos(oracle, N, nranks):
    """Row-block slabs + halo lines (the multi-GPU decomposition) reproduce
    the single-grid operator bit for bit."""
    import gmres_amd.solver as S

    rng = np.random.default_rng(7)
    x = rng.standard_normal(N * N)
    ref = oracle.stvec(x, N)
    X = x.reshape(N, N)  # [j][i]
    for line0, nl in S.slab_partition(N, nranks):
        xs = _dev(X[line0:line0 + nl].reshape(-1))
        lo = _dev(X[line0 - 1]) if line0 > 0 else None
        hi = _dev(X[line0 + nl]) if line0 + nl < N else None
        ys = torch.empty_like(xs)
        S.poisson5(xs, ys, N, nlines=nl, halo_lo=lo, halo_hi=hi)
        torch.cuda.synchronize()
        assert np.array_equal(ys.cpu().numpy(), ref[line0 * N:(line0 + nl) * N])


PREC_CASES = [("cbpr2", 1), ("identity", 1)] + [("cheb", k) for k in range(1, 9)] + [("cheb", 11), ("cheb", 16)]


@pytest.mark.parametrize("N", [16, 64, 126, 128, 129, 130, 256, 372])
@pytest.mark.parametrize("kind,degree", PREC_CASES)
def test_precond_bitexact(oracle, N, kind, degree):
    """Every Chebyshev degree 1..8: ONE temporal-blocked pass of L = k levels
    (k <= CF_LMAX = 8) when N is even; degrees 11 and 16 run two passes (8 + 3,
    8 + 8: the (d, res, z) hand-over).  N < 128 is the one-window SMALL variant
    (lanes beyond N held at zero), 128 one window whose both edges are the
    grid's, 130 / 256 / 372 two to four windows (the last one aligned to the
    grid's E edge, overlapping its neighbour's halo) and more than one line
    tile; odd N takes the per-sweep kernels."""
    import gmres_amd.solver as S

    rng = np.random.default_rng(N + degree)
    r = rng.standard_normal(N * N)
    rd = _dev(r)
    zd = torch.empty_like(rd)
    scratch = torch.empty(3 * N * N, dtype=torch.float64, device="cuda")
    S.precond_apply(rd, zd, N, kind=kind, params=(8.2, 0.2), degree=degree, scratch=scratch)
    torch.cuda.synchronize()
    kid = {"cbpr2": oracle.PREC_CBPR2, "cheb": oracle.PREC_CHEB, "identity": oracle.PREC_IDENTITY}[kind]
    ref = oracle.precond(kid, r, N, params=(8.2, 0.2), degree=degree)
    assert np.array_equal(zd.cpu().numpy(), ref)


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 4097, 1 << 20, (1 << 20) + 3])
def test_dot_and_project(n):
    import gmres_amd.solver as S

    rng = np.random.default_rng(n)
    a = rng.standard_normal(n)
    b = rng.standard_normal(n)
    ad, bd = _dev(a), _dev(b)
    res = torch.zeros(1, dtype=torch.float64, device="cuda")
    S.dot(ad, bd, res)
    torch.cuda.synchronize()
    ref = float(np.dot(a, b))
    scale = float(np.abs(a * b).sum())
    assert abs(res.item() - ref) <= 1e-13 * scale + 1e-300
    # fused MGS projection: h = <w, v>, w -= h v
    S.mgs_project(ad, bd, res)
    torch.cuda.synchronize()
    h = res.item()
    assert abs(h - ref) <= 1e-13 * scale + 1e-300
    w_ref = a - h * b  # same h, same elementwise rounding
    assert np.array_equal(ad.cpu().numpy(), w_ref)


def test_unaligned_pointer_rejected():
    import gmres_amd.solver as S
    from gmres_amd._native import GkError

    x = torch.zeros(65, dtype=torch.float64, device="cuda")
    with pytest.raises(GkError):
        S.dot(x[1:], x[1:], x[:1])


def _ctx_col(c, k):
    """V(:,k+1) of a context, through the device vector API (copy to x)."""
    from gmres_amd import _native as nat

    nat.check(nat.hip().gk_vec_lincomb(c.handle, 0, 0, 2 + k, 0, 0, 0.0, 0.0), "gk_vec_lincomb")
    return c.get_x()


@pytest.mark.parametrize("N,degree", [(130, 3), (256, 6), (256, 8), (1024, 8), (4096, 8)])
def test_fused_chebyshev_norm_epilogue(oracle, N, degree):
    """The ACC_NORM last pass (cycle start: w = M^-1 b, beta = ||w||, V(:,1) = w/beta):
    w is bit-exact, so V(:,1) equals oracle_w / beta_gpu bit for bit, and beta is
    the oracle's norm to summation-order noise -- with the fused passes and the
    per-sweep kernels alike (GK_TUNE_CHEB_FUSED = 6)."""
    import gmres_amd as ga

    w = oracle.precond(oracle.PREC_CHEB, oracle.rhs_ones(N), N, params=(8.2, 0.2), degree=degree)
    bref = float(np.sqrt(np.sum(w * w)))
    for fused in (1, 0):
        with ga.Context(N, 10) as c:
            c.tune(6, fused)
            c.tune(8, 0)  # launch path: the cycle start is the same either way
            c.set_precond("cheb", (8.2, 0.2), degree)
            c.set_rhs_ones()
            beta = c.mgs_cycle_start()
            v1 = _ctx_col(c, 0)
        assert beta == pytest.approx(bref, rel=1e-14)
        assert np.array_equal(v1, w / beta)


@pytest.mark.parametrize("N,degree", [(130, 5), (256, 8), (1024, 8), (2048, 8), (4096, 8)])
def test_fused_chebyshev_dot_epilogue_step(N, degree):
    """The ACC_DOT last pass inside an Arnoldi step (w = M^-1 A V(:,j) fused with
    <w, V(:,1)>): fused passes vs per-sweep kernels give the same Hessenberg
    columns and Krylov vectors for steps 1..4 up to the dot's summation order
    (the two paths reduce over different workgroup grids, so the last bit of a
    dot may differ; the element-wise w is bit-identical, test above)."""
    import gmres_amd as ga

    res = {}
    for fused in (1, 0):
        with ga.Context(N, 10) as c:
            c.tune(6, fused)
            c.set_precond("cheb", (8.2, 0.2), degree)
            c.set_rhs_ones()
            c.mgs_cycle_start()
            cols = [c.mgs_step(j) for j in range(1, 5)]
            res[fused] = (cols, _ctx_col(c, 4))
    for a, b in zip(res[1][0], res[0][0]):
        assert np.allclose(a, b, rtol=1e-12, atol=1e-15)
    assert np.allclose(res[1][1], res[0][1], rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("N,degree", [(130, 5), (1024, 8), (4096, 8)])
def test_fused_stencil_stage_matches_stencil_launch(N, degree):
    """GK_TUNE_CHEB_STEN: the Arnoldi step's Chebyshev pass forming z = A v in
    its stage 0 (no stencil launch) against the stencil launch + pass: the
    element-wise w is the same arithmetic, so the Hessenberg columns and
    Krylov vectors of steps 1..4 agree up to the fused dot's summation order
    (the stage-0 pass has a wider halo, hence another window grid)."""
    import gmres_amd as ga
    from gmres_amd import _native as nat

    res = {}
    for sten in (1, 0):
        with ga.Context(N, 10) as c:
            c.tune(nat.GK_TUNE_CHEB_STEN, sten)
            c.set_precond("cheb", (8.2, 0.2), degree)
            c.set_rhs_ones()
            c.mgs_cycle_start()
            cols = [c.mgs_step(j) for j in range(1, 5)]
            res[sten] = (cols, _ctx_col(c, 4))
    for a, b in zip(res[1][0], res[0][0]):
        assert np.allclose(a, b, rtol=1e-12, atol=1e-15)
    assert np.allclose(res[1][1], res[0][1], rtol=1e-10, atol=1e-14)
