"""Python-side handle on the MI355X GMRES(m) inner cycle.

The solve loops themselves run in the Fortran host (libgmres_fhost.so:
gmres_mgsr_hip_run / gmres_hh_hip_run, which mirror gmres_mgsr_omp /
gmres_mgsr_mf / gmres_hh_omp / gmres_hh_prec_omp of the reference) on top of
the HIP C-ABI (libgmres_hip.so).  This module only owns the device context
(one per GPU / rank), sets the right-hand side and the preconditioner, and
marshals arrays -- the "harness" role the reference's test drivers play
(tests/test_poisson_mf.f90).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _native as nat

PREC = {"identity": nat.GK_PREC_IDENTITY, "none": nat.GK_PREC_IDENTITY,
        "cbpr2": nat.GK_PREC_CBPR2, "cheb": nat.GK_PREC_CHEB, "chebyshev": nat.GK_PREC_CHEB}
MGSR_MF, MGSR_OMP = 0, 1


def _p(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(nat._dp)


def slab_partition(N: int, nranks: int) -> list[tuple[int, int]]:
    """Row-block decomposition over the slow grid index j:
    rank r owns grid lines [line0_r, line0_r + nlines_r), contiguous, the
    first N % nranks ranks one line more.  Every rank's slice of every vector
    (and of every Krylov column) is then contiguous in Fortran order."""
    if nranks < 1 or nranks > N:
        raise ValueError(f"cannot split {N} grid lines over {nranks} ranks")
    base, extra = divmod(N, nranks)
    out, l0 = [], 0
    for r in range(nranks):
        nl = base + (1 if r < extra else 0)
        out.append((l0, nl))
        l0 += nl
    return out


class LocalGroup:
    """In-process communicator (include/gmres_hip.h gk_group): several
    contexts of one process, one host thread per rank, RCCL's message pattern."""

    def __init__(self, nranks: int):
        h = nat.c_vp()
        nat.check(nat.hip().gk_group_create(int(nranks), ctypes.byref(h)), "gk_group_create")
        self._h, self.nranks = h, int(nranks)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            nat.hip().gk_group_destroy(self._h)
            self._h = None


@dataclass
class SolveResult:
    x: np.ndarray            # local slab of the solution
    final_err: np.ndarray    # final_err(1:m) of the last cycle
    v_err: np.ndarray        # v_err(1:m+1)
    n_out: int
    cycles_out: int          # restart_out / stages_out
    n_cycles: int
    m: int
    hist_res: np.ndarray = field(default_factory=lambda: np.zeros(0))
    hist_ferr: np.ndarray = field(default_factory=lambda: np.zeros((0, 0)))

    @property
    def iterations(self) -> int:
        """(stages-1)*m + n_out, as tests/test_poisson_mf.f90:47 reports it."""
        return (self.cycles_out - 1) * self.m + self.n_out


class Context:
    """One device context: a slab of grid lines of an N x N Poisson problem on
    one GPU, with Krylov dimension m."""

    def __init__(self, N: int, m: int, device: int = 0, line0: int = 0, nlines: int | None = None):
        self.N, self.m, self.device = int(N), int(m), int(device)
        self.line0 = int(line0)
        self.nlines = int(N if nlines is None else nlines)
        self.nranks, self.rank = 1, 0
        h = nat.c_vp()
        nat.check(nat.hip().gk_create(self.device, self.N, self.line0, self.nlines, self.m, ctypes.byref(h)),
                  "gk_create")
        self._h = h
        n = nat.c_ll()
        nat.check(nat.hip().gk_local_size(self._h, ctypes.byref(n)), "gk_local_size")
        self.nloc = int(n.value)

    # -- lifetime --------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            nat.hip().gk_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # -- multi-GPU -----------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        nat.check(nat.hip().gk_comm_unique_id(buf), "gk_comm_unique_id")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, max_lines: int, uid: bytes) -> None:
        assert len(uid) == 128
        nat.check(nat.hip().gk_comm_init(self._h, nranks, rank, max_lines, uid), "gk_comm_init")
        self.nranks, self.rank = nranks, rank

    def comm_init_local(self, group: "LocalGroup", rank: int, max_lines: int) -> None:
        nat.check(nat.hip().gk_comm_init_local(self._h, group.handle, rank, max_lines), "gk_comm_init_local")
        self.nranks, self.rank = group.nranks, rank
        self._group = group  # keep alive

    # --- device exchange ("xgmi" collective back-end, gmres_hip.h) ---
    def comm_init_xgmi(self, nranks: int, rank: int, max_lines: int) -> None:
        """Slab decomposition without RCCL; collectives by device exchange
        once xchg_open() has mapped every rank's receive region."""
        nat.check(nat.hip().gk_comm_init_xgmi(self._h, nranks, rank, max_lines), "gk_comm_init_xgmi")
        self.nranks, self.rank = nranks, rank

    def xchg_handle(self) -> bytes:
        buf = ctypes.create_string_buffer(64)
        nat.check(nat.hip().gk_xchg_handle(self._h, buf), "gk_xchg_handle")
        return buf.raw

    def xchg_open(self, handles: list[bytes]) -> None:
        assert len(handles) == self.nranks and all(len(h) == 64 for h in handles)
        nat.check(nat.hip().gk_xchg_open(self._h, b"".join(handles)), "gk_xchg_open")

    def xchg_local(self) -> None:
        nat.check(nat.hip().gk_xchg_local(self._h), "gk_xchg_local")

    def xchg_enable(self, on: bool) -> None:
        nat.check(nat.hip().gk_xchg_enable(self._h, int(bool(on))), "gk_xchg_enable")

    def comm_info(self) -> dict:
        """The collective back-end actually in use and the rank count its
        communicator reports (gk_comm_info)."""
        k, nr = ctypes.c_int(), ctypes.c_int()
        nat.check(nat.hip().gk_comm_info(self._h, ctypes.byref(k), ctypes.byref(nr)), "gk_comm_info")
        return {"kind": nat.COMM_KINDS.get(k.value, k.value), "nranks": nr.value}

    def comm_latency(self, iters: int = 200) -> dict:
        """Collective (all ranks): mean us of one partial-slab all-reduce and
        one halo exchange through the collective in use (gk_comm_latency)."""
        a, h = ctypes.c_double(), ctypes.c_double()
        nat.check(nat.hip().gk_comm_latency(self._h, iters, ctypes.byref(a), ctypes.byref(h)), "gk_comm_latency")
        return {"allreduce_us": a.value, "halo_us": h.value}

    def xchg_selftest(self, timeout_ms: int = 5000) -> bool:
        """Collective self-test of the device exchange; False (and the
        exchange disabled on this rank) when it fails."""
        rc = nat.hip().gk_xchg_selftest(self._h, int(timeout_ms))
        if rc == nat.GK_ERR_COMM:
            self.xchg_error = nat.last_error()
            return False
        nat.check(rc, "gk_xchg_selftest")
        return True

    # -- problem setup ---------------------------------------------------
    def set_precond(self, kind: str | int = "identity", params=(8.2, 0.2), degree: int = 8) -> None:
        k = PREC[kind] if isinstance(kind, str) else int(kind)
        pr = np.ascontiguousarray(params, dtype=np.float64)
        nat.check(nat.hip().gk_set_precond(self._h, k, _p(pr), pr.size, int(degree)), "gk_set_precond")

    def set_rhs(self, b_local: np.ndarray) -> None:
        b = np.ascontiguousarray(b_local, dtype=np.float64).reshape(-1)
        assert b.size == self.nloc
        nat.check(nat.hip().gk_set_rhs(self._h, _p(b)), "gk_set_rhs")

    def set_rhs_ones(self) -> None:
        """b = A*1, the manufactured RHS of every reference driver."""
        nat.check(nat.hip().gk_set_rhs_ones(self._h), "gk_set_rhs_ones")

    def rhs_norm(self) -> float:
        v = ctypes.c_double()
        nat.check(nat.hip().gk_rhs_norm(self._h, ctypes.byref(v)), "gk_rhs_norm")
        return v.value

    def get_x(self) -> np.ndarray:
        x = np.empty(self.nloc)
        nat.check(nat.hip().gk_get_x(self._h, _p(x)), "gk_get_x")
        return x

    def get_basis(self, col: int, which: int = 0) -> np.ndarray:
        """Column col (0-based) of the device basis: which 0 = V (Krylov basis
        or Householder reflectors), 1 = the basis gk_hh_verr rebuilt."""
        v = np.empty(self.nloc, dtype=np.float64)
        nat.check(nat.hip().gk_get_basis(self._h, which, col, _p(v)), "gk_get_basis")
        return v

    def set_x(self, x: np.ndarray) -> None:
        xx = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
        nat.check(nat.hip().gk_set_x(self._h, _p(xx)), "gk_set_x")

    def zero_x(self) -> None:
        nat.check(nat.hip().gk_zero_x(self._h), "gk_zero_x")

    def apply(self, v: np.ndarray, what: int = 0) -> np.ndarray:
        """what = 0: A v ; what = 1: M^-1 v (host arrays, local slab)."""
        vin = np.ascontiguousarray(v, dtype=np.float64).reshape(-1)
        out = np.empty(self.nloc)
        nat.check(nat.hip().gk_apply(self._h, what, _p(vin), _p(out)), "gk_apply")
        return out

    def true_residual(self) -> float:
        v = ctypes.c_double()
        nat.check(nat.hip().gk_true_residual(self._h, ctypes.byref(v)), "gk_true_residual")
        return v.value

    def lanczos_bounds(self, k: int = 40) -> tuple[float, float]:
        """Extreme Ritz values of A after k Lanczos steps (spectrum estimate
        for the Chebyshev preconditioner interval)."""
        lo, hi = ctypes.c_double(), ctypes.c_double()
        nat.check(nat.hip().gk_lanczos_bounds(self._h, int(k), ctypes.byref(lo), ctypes.byref(hi)),
                  "gk_lanczos_bounds")
        return lo.value, hi.value

    # -- Arnoldi pieces (for tests / custom drivers) -----------------------
    def mgs_cycle_start(self) -> float:
        v = ctypes.c_double()
        nat.check(nat.hip().gk_mgs_cycle_start(self._h, ctypes.byref(v)), "gk_mgs_cycle_start")
        return v.value

    def mgs_step(self, j: int) -> np.ndarray:
        h = np.zeros(j + 1)
        nat.check(nat.hip().gk_mgs_step(self._h, j, _p(h)), "gk_mgs_step")
        return h

    def update_x(self, y: np.ndarray) -> None:
        yy = np.ascontiguousarray(y, dtype=np.float64)
        nat.check(nat.hip().gk_update_x(self._h, _p(yy), yy.size), "gk_update_x")

    # -- profiling -------------------------------------------------------
    def profile(self, enable: bool = True) -> None:
        nat.check(nat.hip().gk_profile_enable(self._h, int(enable)), "gk_profile_enable")

    def profile_reset(self) -> None:
        nat.check(nat.hip().gk_profile_reset(self._h), "gk_profile_reset")

    def profile_read(self) -> dict:
        out = {}
        for kid, name in enumerate(nat.KID_NAMES):
            ms = ctypes.c_double()
            n = nat.c_ll()
            nat.check(nat.hip().gk_profile_read(self._h, kid, ctypes.byref(ms), ctypes.byref(n)),
                      "gk_profile_read")
            out[name] = (ms.value, int(n.value))
        return out

    def res_split(self, mode: int = -1, which: int = 0) -> dict:
        """In-launch time split of the resident launches (gk_profile_res_split):
        mode 1 enable + zero, 2 zero, 0 disable, -1 read only; which 0 MGS-R
        steps, 1 Householder UP chains, 2 Householder DOWN chains."""
        p, w, t = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = nat.c_ll()
        nat.check(nat.hip().gk_profile_res_split(self._h, int(mode), int(which), ctypes.byref(p), ctypes.byref(w),
                                                 ctypes.byref(t), ctypes.byref(n)), "gk_profile_res_split")
        return {"pass_ms": p.value, "wait_ms": w.value, "total_ms": t.value, "launches": int(n.value)}

    def res_split_wg(self, which: int = 0) -> tuple[np.ndarray, np.ndarray]:
        """Per-workgroup pass / wait ms of the resident launches (gk_profile_res_wg)."""
        p = np.zeros(1024)
        w = np.zeros(1024)
        n = ctypes.c_int()
        nat.check(nat.hip().gk_profile_res_wg(self._h, int(which), _p(p), _p(w), 1024, ctypes.byref(n)),
                  "gk_profile_res_wg")
        return p[: n.value], w[: n.value]

    def res_trace(self, arm: int, j: int = 0, mode: int = 0):
        """All-gather trace of one resident launch (gk_profile_res_trace): arm 1 traces the
        MGS-R step launches of step j (mode 0), 0 stops; -1 returns
        (publish, seen) wall-clock ms as two [workgroups, exchanges] arrays."""
        if arm != -1:
            nat.check(nat.hip().gk_profile_res_trace(self._h, int(arm), int(j), int(mode), None, 0, 0, None, None,
                                                     None), "gk_profile_res_trace")
            return None
        maxwg, maxx = 1024, 1026
        buf = np.zeros(maxwg * maxx * 2, dtype=np.uint64)
        g, x, tpm = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        nat.check(nat.hip().gk_profile_res_trace(self._h, -1, 0, 0, buf.ctypes.data, maxwg, maxx, ctypes.byref(g),
                                                 ctypes.byref(x), ctypes.byref(tpm)), "gk_profile_res_trace")
        t = buf[: g.value * x.value * 2].reshape(g.value, x.value, 2).astype(np.float64)
        t0 = t[t > 0].min() if np.any(t > 0) else 0.0
        return (t[:, :, 0] - t0) / tpm.value, (t[:, :, 1] - t0) / tpm.value

    def res_info(self, hh: bool = False) -> dict:
        """The resident-step plan this context uses now (gk_res_info): variant
        name (None = launch per projection), workgroups, chunk split."""
        return _res_dict(lambda buf: nat.hip().gk_res_info(self._h, int(hh), buf), "gk_res_info")

    def tune(self, key: int, value: int) -> None:
        """Launch-policy knob (include/gmres_hip.h GK_TUNE_*)."""
        nat.check(nat.hip().gk_set_tuning(self._h, int(key), int(value)), "gk_set_tuning")

    def sync(self) -> None:
        nat.check(nat.hip().gk_sync(self._h), "gk_sync")

    def debug_hold_stream(self, hold: bool) -> None:
        """Test hook (gk_debug_hold_stream): hold the context's stream behind a
        never-written mapped word, or release it."""
        nat.check(nat.hip().gk_debug_hold_stream(self._h, int(hold)), "gk_debug_hold_stream")


def _res_dict(call, what: str) -> dict:
    buf = (nat.c_ll * len(nat.RES_INFO_KEYS))()
    nat.check(call(buf), what)
    d = dict(zip(nat.RES_INFO_KEYS, (int(v) for v in buf)))
    d["variant"] = nat.RES_VARIANTS[d["variant"]]
    return d


def res_plan_query(nloc: int, cus: int = 256, share: int = 1, hh: bool = False, nt: int = -1,
                   block: int = 1) -> dict:
    """The resident-step variant a slab of nloc local unknowns selects on a
    device of `cus` compute units shared by `share` contexts, with the MGS step's
    projection block `block` (GK_TUNE_RES_BLOCK; gk_res_plan_query: host-only, no
    GPU touched)."""
    return _res_dict(lambda buf: nat.hip().gk_res_plan_query(int(nloc), int(cus), int(share), int(hh), int(nt),
                                                             int(block), buf),
                     "gk_res_plan_query")


def _alloc_hist(m: int, max_cycles: int, want_hist: bool):
    if want_hist:
        return np.zeros(max_cycles), np.zeros(max_cycles * m)
    return np.zeros(1), np.zeros(1)


def gmres_mgsr(ctx: Context, tol: float = 1e-15, variant: int = MGSR_OMP, max_cycles: int = 1000,
               want_verr: bool = True, want_hist: bool = False, want_x: bool = True) -> SolveResult:
    """Restarted MGS-R GMRES(m) from x0 = 0 (Fortran host loop, HIP vector work).
    variant MGSR_OMP = gmres_mgsr_omp semantics, MGSR_MF = gmres_mgsr_mf.
    want_x = False: the solution stays in HBM (result x empty; ctx.get_x() later)."""
    m = ctx.m
    x = np.zeros(ctx.nloc if want_x else 1)
    fe = np.zeros(m)
    ve = np.zeros(m + 1)
    n_out, ro, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    hr, hf = _alloc_hist(m, max_cycles, want_hist)
    st = nat.fhost().gmres_mgsr_hip_run(ctx.handle, m, tol, variant, max_cycles, _p(x), _p(fe), _p(ve),
                                        ctypes.byref(n_out), ctypes.byref(ro), int(want_verr), int(want_hist),
                                        _p(hr), _p(hf), ctypes.byref(nc), int(not want_x))
    nat.check(st, "gmres_mgsr_hip_run")
    r = SolveResult(x=x if want_x else np.zeros(0), final_err=fe, v_err=ve, n_out=n_out.value, cycles_out=ro.value, n_cycles=nc.value, m=m)
    if want_hist:
        r.hist_res = hr[: nc.value].copy()
        r.hist_ferr = hf.reshape(max_cycles, m)[: nc.value].copy()
    return r


def gmres_hh(ctx: Context, tol: float = 1e-15, precondition: bool = False, midcycle_exit: bool | None = None,
             max_cycles: int = 1000, want_verr: bool = True, want_hist: bool = False,
             want_x: bool = True) -> SolveResult:
    """Householder GMRES(m): precondition=False -> gmres_hh_omp (full cycles);
    precondition=True -> gmres_hh_prec_omp (in-cycle convergence latch).
    want_x = False: the solution stays in HBM (result x empty; ctx.get_x() later)."""
    if midcycle_exit is None:
        midcycle_exit = precondition
    m = ctx.m
    x = np.zeros(ctx.nloc if want_x else 1)
    fe = np.zeros(m)
    ve = np.zeros(m + 1)
    n_out, so, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    hr, hf = _alloc_hist(m, max_cycles, want_hist)
    st = nat.fhost().gmres_hh_hip_run(ctx.handle, m, tol, int(precondition), int(midcycle_exit), max_cycles,
                                      _p(x), _p(fe), _p(ve), ctypes.byref(n_out), ctypes.byref(so),
                                      int(want_verr), int(want_hist), _p(hr), _p(hf), ctypes.byref(nc),
                                      int(not want_x))
    nat.check(st, "gmres_hh_hip_run")
    r = SolveResult(x=x if want_x else np.zeros(0), final_err=fe, v_err=ve, n_out=n_out.value, cycles_out=so.value, n_cycles=nc.value, m=m)
    if want_hist:
        r.hist_res = hr[: nc.value].copy()
        r.hist_ferr = hf.reshape(max_cycles, m)[: nc.value].copy()
    return r


def _short(solver: int, ctx: Context, tol: float, max_iter: int, want_hist: bool, fused: bool):
    if ctx.m < 8:
        raise ValueError("short-recurrence solvers need a context with m >= 8 (scratch vectors)")
    it = ctypes.c_int(max_iter)
    res = ctypes.c_double()
    hist = np.zeros(max(max_iter, 1) if want_hist else 1)
    fh = nat.fhost()
    if fused:
        name = "pcg_hip_run" if solver == nat.GK_SR_PCG else "pbicgstab_hip_run"
        st = getattr(fh, name)(ctx.handle, tol, ctypes.byref(it), ctypes.byref(res), int(want_hist), _p(hist))
    else:
        name = "sr_hip_run_seq"
        st = fh.sr_hip_run_seq(ctx.handle, solver, tol, ctypes.byref(it), ctypes.byref(res), int(want_hist),
                               _p(hist))
    nat.check(st, name)
    x = ctx.get_x()
    return x, it.value, res.value, (hist[: np.count_nonzero(hist)].copy() if want_hist else None)


def pcg(ctx: Context, tol: float = 1e-9, max_iter: int = 1000, want_hist: bool = False, fused: bool = True):
    """pcg_omp (src/cg.f90:154-234) on the device: (x, iter, res, hist).
    fused = True: the fused passes with the scalars on the device (gk_sr_*);
    False: the reference's operation sequence, one device call per BLAS-1 op."""
    return _short(nat.GK_SR_PCG, ctx, tol, max_iter, want_hist, fused)


def pbicgstab(ctx: Context, tol: float = 1e-9, max_iter: int = 1000, want_hist: bool = False, fused: bool = True):
    """pbicgstab_omp (src/bicgstab.f90:91-182) on the device: (x, iters, res, hist); fused as in pcg."""
    return _short(nat.GK_SR_BICGSTAB, ctx, tol, max_iter, want_hist, fused)


class SrSolve:
    """Direct handle on the fused short-recurrence passes (gk_sr_*): start a
    solve, queue iterations, read the device status -- what bench.py times."""

    def __init__(self, ctx: Context, solver: str, tol: float, max_iter: int):
        self.ctx = ctx
        self.solver = {"pcg": nat.GK_SR_PCG, "pbicgstab": nat.GK_SR_BICGSTAB}[solver]
        nat.check(nat.hip().gk_sr_start(ctx.handle, self.solver, tol, max_iter), "gk_sr_start")

    def iterate(self, k: int) -> None:
        nat.check(nat.hip().gk_sr_iterate(self.ctx.handle, k), "gk_sr_iterate")

    def status(self, wait_all: bool = True) -> tuple[int, int, float]:
        ex, dn, res = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        nat.check(nat.hip().gk_sr_status(self.ctx.handle, int(wait_all), ctypes.byref(ex), ctypes.byref(dn),
                                         ctypes.byref(res)), "gk_sr_status")
        return ex.value, dn.value, res.value

    def history(self, n: int) -> np.ndarray:
        h = np.zeros(max(n, 1))
        nat.check(nat.hip().gk_sr_history(self.ctx.handle, _p(h), n), "gk_sr_history")
        return h[:n]


# ---------------------------------------------------------------- kernels ---
# Stateless kernel-level calls on caller-owned device memory (torch tensors on
# cuda: plumbing only).  Used by the kernel parity tests.

def _stream_handle(stream) -> int:
    return int(stream.cuda_stream) if stream is not None else 0


def poisson5(x, y, N: int, nlines: int | None = None, halo_lo=None, halo_hi=None, stream=None) -> None:
    nl = N if nlines is None else nlines
    nat.check(nat.hip().gk_poisson5(N, nl, x.data_ptr(), halo_lo.data_ptr() if halo_lo is not None else None,
                                    halo_hi.data_ptr() if halo_hi is not None else None, y.data_ptr(),
                                    _stream_handle(stream)), "gk_poisson5")


def precond_apply(r, z, N: int, kind: str = "cbpr2", params=(8.2, 0.2), degree: int = 8, scratch=None,
                  stream=None) -> None:
    pr = np.ascontiguousarray(params, dtype=np.float64)
    nat.check(nat.hip().gk_precond_apply(N, PREC[kind], _p(pr), degree, r.data_ptr(), z.data_ptr(),
                                         scratch.data_ptr() if scratch is not None else None,
                                         _stream_handle(stream)), "gk_precond_apply")


def mgs_project(w, va, result, stream=None) -> None:
    nat.check(nat.hip().gk_mgs_project(w.numel(), w.data_ptr(), va.data_ptr(), result.data_ptr(),
                                       _stream_handle(stream)), "gk_mgs_project")


def dot(a, b, result, stream=None) -> None:
    nat.check(nat.hip().gk_dot(a.numel(), a.data_ptr(), b.data_ptr(), result.data_ptr(), _stream_handle(stream)),
              "gk_dot")
