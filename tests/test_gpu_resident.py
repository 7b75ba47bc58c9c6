"""Resident MGS-R step (gk::k_mgs_res, include/gmres_hip.h GK_TUNE_RES): the whole
cascade of an Arnoldi step (gmres_mgsr.f90:341-363, :384) in ONE persistent launch,
w and the running Krylov column held in registers, the dots all-gathered inside the
launch.

Parity: the element-wise arithmetic is the launch path's (k_proj / k_scale), only the
dot summation order differs, so the per-cycle true residuals must agree with the
launch-per-projection path to reduction-order noise and with the CPU oracle within the
reference's own tolerance.  The variants cover: fully resident with the
next column prefetched (R2 2/4/8), two-array residency (R2 16), a partly streamed
vector (cap below the vector size, few workgroups), odd N (tail element), every
preconditioner.  Determinism: two runs give bit-identical histories.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T_RES, T_R2, T_SHARE, T_TMO = 8, 9, 10, 11


def _run(N, m, prec, res, r2=0, share=1, cycles=4, degree=4, want_prof=False, wonly=-1, method="mgsr",
         hh_fuse=1, pc=-1):
    import gmres_amd as ga

    with ga.Context(N, m) as c:
        c.tune(21, pc)  # GK_TUNE_RES_PC
        c.tune(T_RES, res)
        c.tune(15, hh_fuse)  # GK_TUNE_HH_FUSE
        c.tune(13, wonly)  # GK_TUNE_RES_WONLY
        c.tune(T_R2, r2)
        c.tune(T_SHARE, share)
        c.tune(T_TMO, 5000)
        c.set_precond(prec, (8.2, 0.2), degree)
        c.set_rhs_ones()
        if want_prof:
            c.profile(True)
            c.profile_reset()
        if method == "hh":
            r = ga.gmres_hh(c, 1e-15, precondition=(prec != "identity"), max_cycles=cycles, want_hist=True)
        else:
            r = ga.gmres_mgsr(c, 1e-15, max_cycles=cycles, want_hist=True)
        prof = c.profile_read() if want_prof else None
        r.variant = c.res_info(hh=method == "hh")["variant"]
    return r, prof


CASES = [
    # N, m, prec, r2 cap, share (workgroups = CUs / share)
    (64, 20, "identity", 0, 1),      # fully resident, R2 = 2, prefetch
    (130, 30, "cbpr2", 2, 8),        # 32 workgroups x 512 x 2 < n/2: streamed tail of the vector
    (45, 12, "identity", 2, 64),     # odd N: the tail element, 4 workgroups
    (256, 40, "cheb", 12, 16),       # two-array variant (+ LDS-resident w)
    (200, 25, "identity", 4, 32),    # R2 = 4 with a streamed part
    (512, 30, "identity", 8, 4),     # R2 = 8, fully resident
    # even spread of the resident chunks (ResPlan::r2e / l2e): register part and
    # LDS part only partly used, as at 2048^2 with every CU
    (1024, 10, "identity", 0, 2),    # auto variant, 128 workgroups
    (700, 12, "cbpr2", 12, 4),       # two-array variant, LDS part partly filled
    (2048, 8, "identity", 0, 1),     # the size whose contiguous fill idled 70 % of the workgroups
]


WCASES = [  # w-only variant (one wave per SIMD): few workgroups so the LDS and streamed parts are used
    (300, 20, "identity", 12, 64),
    (181, 16, "cbpr2", 12, 128),     # odd N
    (512, 24, "cheb", 12, 32),
]


PCASES = [  # column-cache variant (k_mgs_wpc, 512 threads), forced: cached registers + LDS, uncached, streamed
    (300, 20, "identity", 0, 64),    # 4 workgroups x 22 chunks (4 in registers, 18 in LDS), a streamed tail
    (181, 16, "cbpr2", 0, 128),      # odd N (tail element), 2 x 16 chunks
    (512, 24, "cheb", 0, 32),        # 8 workgroups x 32 chunks: exactly the 4096^2 / 2 share (9 uncached)
]


@pytest.mark.parametrize("N,m,prec,r2,share,wonly,pc", [c + (-1, -1) for c in CASES] + [c + (1, 0) for c in WCASES]
                         + [c + (-1, 1) for c in PCASES])
def test_resident_matches_launch_path(N, m, prec, r2, share, wonly, pc):
    ref, _ = _run(N, m, prec, res=0)
    got, prof = _run(N, m, prec, res=1, r2=r2, share=share, want_prof=True, wonly=wonly, pc=pc)
    if pc == 1:
        assert got.variant == "w+column", got.variant
    # the resident kernel ran every step (k_proj only in the off-cycle diagnostics)
    assert prof["res"][1] > 0 and prof["proj"][1] < prof["res"][1] // 4, prof
    assert got.n_cycles == ref.n_cycles
    h, r = got.hist_res, ref.hist_res
    tol = np.where(r > 1e-8, 1e-10, 1e-4)
    assert np.all(np.abs(h - r) <= tol * r + 1e-16), (h, r)
    k = min(got.n_out, ref.n_out)
    assert np.allclose(got.final_err[:k], ref.final_err[:k], rtol=1e-6, atol=1e-16)


@pytest.mark.parametrize("N,m,prec", [(128, 30, "identity"), (128, 30, "cbpr2")])
def test_resident_vs_oracle_to_convergence(oracle, N, m, prec):
    """Config 1 shape to tol 1e-15 on the resident path, against the oracle
    (reference restatement) with the reference-derived tolerance."""
    got, _ = _run(N, m, prec, res=1, cycles=1000)
    kind = {"identity": oracle.PREC_IDENTITY, "cbpr2": oracle.PREC_CBPR2}[prec]
    ref = oracle.gmres_mgsr(oracle.rhs_ones(N), N, m, prec=kind, variant=oracle.MGSR_OMP)
    assert abs(got.iterations - ref.iterations) <= max(1, 0.01 * ref.iterations)
    k = min(len(got.hist_res), len(ref.hist_res))
    dev = np.abs(got.hist_res[:k] - ref.hist_res[:k])
    assert np.all(dev <= 1e-5 * ref.hist_res[:k] + 1e-13)
    assert np.max(np.abs(got.x - 1.0)) < 1e-9


def test_resident_is_deterministic():
    a, _ = _run(96, 24, "cbpr2", res=1, r2=2, share=16, cycles=3)
    b, _ = _run(96, 24, "cbpr2", res=1, r2=2, share=16, cycles=3)
    assert np.array_equal(a.hist_res, b.hist_res)
    assert np.array_equal(a.x, b.x)


def test_resident_1024_vs_reference():
    """Config 2 size: the reference's own per-cycle true residuals (serial run)."""
    import json
    import os

    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_known_answers.json")))
    g = gold["mgsr_identity_1024_m95"]["cycle_true_residual"]
    got, prof = _run(1024, 95, "identity", res=1, cycles=3, want_prof=True)
    assert prof["res"][1] > 0
    assert np.allclose(got.hist_res, g[: len(got.hist_res)], rtol=1e-9, atol=0.0)


# Householder steps as resident reflection chains (gk::RES_HH_DOWN: v_j = P_1..P_j e_j,
# gmres_hh.f90:269-283; gk::RES_HH_UP: w = P_j..P_1 A v_j + ||w(j+1:n)||^2, :290-305), in
# every variant of the resident kernels.  The reflection arithmetic is k_proj's with
# coef 2 (bit-identical element-wise); only the dot summation order differs.
HCASES = [
    # N, m, prec, r2 cap, share, w-only
    (64, 20, "identity", 0, 1, -1),     # fully resident, R2 = 2, prefetch
    (45, 12, "cbpr2", 2, 64, -1),       # odd N (tail element), streamed part
    (200, 25, "identity", 4, 32, -1),   # R2 = 4 with a streamed part
    (256, 40, "identity", 12, 16, -1),  # two-array variant + LDS-resident w
    (300, 20, "identity", 12, 64, 1),   # w-only: registers + LDS + streamed
    (181, 16, "cbpr2", 12, 128, 1),     # w-only, odd N
]
HPCASES = [  # the column-cache variant's reflection chains (forced)
    (300, 20, "identity", 0, 64, 0),
    (181, 16, "cbpr2", 0, 64, 0),
    (512, 24, "identity", 0, 32, 0),  # the full 32-chunk share: uncached chunks too
]


@pytest.mark.parametrize("N,m,prec,r2,share,wonly,pc", [c + (-1,) for c in HCASES] + [c + (1,) for c in HPCASES])
def test_resident_householder_matches_launch_path(N, m, prec, r2, share, wonly, pc):
    ref, _ = _run(N, m, prec, res=0, method="hh")
    got, prof = _run(N, m, prec, res=1, r2=r2, share=share, want_prof=True, wonly=wonly, method="hh", pc=pc)
    if pc == 1:
        assert got.variant == "w+column", got.variant
    assert prof["res"][1] > 0 and prof["proj"][1] < prof["res"][1] // 4, prof  # k_proj: diagnostics only
    assert got.n_cycles == ref.n_cycles
    h, r = got.hist_res, ref.hist_res
    tol = np.where(r > 1e-6, 1e-9, np.where(r > 1e-12, 1e-3, 5e-2))  # HH tiers (test_gpu_solver)
    assert np.all(np.abs(h - r) <= tol * r + 1e-16), (h, r)


def test_resident_householder_vs_oracle_to_convergence(oracle):
    """Config 1 shape, gmres_hh_omp (full cycles) on the resident path, against the
    oracle with the Householder tiers of test_gpu_solver._hist_close_hh."""
    got, prof = _run(128, 30, "identity", res=1, cycles=1000, want_prof=True, method="hh")
    ref = oracle.gmres_hh(oracle.rhs_ones(128), 128, 30, midcycle_exit=0)
    assert prof["res"][1] > 0
    assert got.iterations == ref.iterations
    k = min(len(got.hist_res), len(ref.hist_res))
    g, r = got.hist_res[:k], ref.hist_res[:k]
    rtol = np.where(r > 1e-6, 1e-8, np.where(r > 1e-12, 1e-3, 5e-2))
    assert np.all(np.abs(g - r) <= rtol * r + 1e-16)
    assert np.max(np.abs(got.x - 1.0)) < 1e-9


@pytest.mark.parametrize("N,m,prec,r2,share", [(300, 20, "identity", 12, 64), (181, 16, "cbpr2", 12, 128),
                                               (512, 30, "identity", 12, 16)])
def test_householder_fused_step_matches_unfused(N, m, prec, r2, share):
    """GK_TUNE_HH_FUSE: with the w-only variant the DOWN chain builds e_j in place (no
    k_set_unit) and the UP chain ends with the reflector fix-up and P(:,j+1) = w/||w||
    (gmres_hh.f90:306-318) instead of k_hh_fix + k_scale.  The element arithmetic is the
    same; only ||w||^2 of the fixed vector is summed in another order, so the histories
    agree to reduction-order noise, and the fused step runs none of the folded launches."""
    ref, pr = _run(N, m, prec, res=1, r2=r2, share=share, want_prof=True, wonly=1, method="hh", hh_fuse=0)
    got, pg = _run(N, m, prec, res=1, r2=r2, share=share, want_prof=True, wonly=1, method="hh", hh_fuse=1)
    assert got.n_cycles == ref.n_cycles and got.iterations == ref.iterations
    h, r = got.hist_res, ref.hist_res
    tol = np.where(r > 1e-6, 1e-10, np.where(r > 1e-12, 1e-4, 5e-2))
    assert np.all(np.abs(h - r) <= tol * r + 1e-16), (h, r)
    k = min(got.n_out, ref.n_out)
    assert np.allclose(got.final_err[:k], ref.final_err[:k], rtol=1e-6, atol=1e-16)
    # per step the unfused path launches k_set_unit + k_hh_fix ("other") and k_scale
    assert pg["scale"][1] < pr["scale"][1] and pg["other"][1] < pr["other"][1], (pg, pr)
