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


@pytest.mark.parametrize("N", [16, 64, 129, 256])
@pytest.mark.parametrize("kind,degree", [("cbpr2", 1), ("cheb", 1), ("cheb", 8), ("identity", 1)])
def test_precond_bitexact(oracle, N, kind, degree):
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
