"""ctypes wrapper for the CPU oracle (oracle/gmres_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg.  The product path (gmres_amd/) never
imports this module.

Every function restates the reference Fortran (AlexanderGSC/gmres) in the same
operation order; see gmres_oracle.c for the file:line map.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

PREC_IDENTITY, PREC_CBPR2, PREC_CHEB = 0, 1, 2
MGSR_MF, MGSR_OMP = 0, 1
PREC_NAMES = {"identity": PREC_IDENTITY, "none": PREC_IDENTITY, "cbpr2": PREC_CBPR2,
              "cheb": PREC_CHEB, "chebyshev": PREC_CHEB}

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_lib = None


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc is in the image)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or (
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "gmres_oracle.c"))
        ):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.or_norm2.restype = ctypes.c_double
        L.or_norm2.argtypes = [_dp, ctypes.c_longlong]
        L.or_dot.restype = ctypes.c_double
        L.or_dot.argtypes = [_dp, _dp, ctypes.c_longlong]
        L.or_stvec.argtypes = [_dp, _dp, ctypes.c_int]
        L.or_precond.argtypes = [ctypes.c_int, _dp, _dp, _dp, _dp, _dp, ctypes.c_int, ctypes.c_int]
        L.or_set_threads.argtypes = [ctypes.c_int]
        L.or_cbpr2_coeffs.argtypes = [_dp, _dp, _dp]
        common = [_dp, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, _dp,
                  ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp, _dp, _ip, _ip, _dp,
                  _dp, _ip, ctypes.c_int, _dp]
        L.or_gmres_mgsr.argtypes = common
        L.or_gmres_mgsr.restype = ctypes.c_int
        L.or_gmres_hh.argtypes = common
        L.or_gmres_hh.restype = ctypes.c_int
        kry = [_dp, ctypes.c_int, ctypes.c_double, _ip, _dp, ctypes.c_int, _dp, ctypes.c_int, _dp, _dp]
        L.or_pcg.argtypes = kry
        L.or_pbicgstab.argtypes = kry
        _lib = L
    return _lib


def _p(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_dp)


def set_threads(nt: int) -> None:
    lib().or_set_threads(int(nt))


def norm2(x: np.ndarray) -> float:
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().or_norm2(_p(x), x.size)


def dot(a: np.ndarray, b: np.ndarray) -> float:
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    return lib().or_dot(_p(a), _p(b), a.size)


def stvec(x: np.ndarray, N: int) -> np.ndarray:
    """y = A x (poisson.f90:33-77); x flat, Fortran column-major, length N*N."""
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    assert x.size == N * N
    y = np.empty_like(x)
    lib().or_stvec(_p(x), _p(y), N)
    return y


def precond(kind: int, r: np.ndarray, N: int, params=(8.2, 0.2), degree: int = 8) -> np.ndarray:
    r = np.ascontiguousarray(r, dtype=np.float64).reshape(-1)
    z = np.empty_like(r)
    aux = np.empty_like(r)
    aux2 = np.empty_like(r)
    pr = np.asarray(params, dtype=np.float64)
    lib().or_precond(kind, _p(r), _p(z), _p(aux), _p(aux2), _p(pr), degree, N)
    return z


def cbpr2_coeffs(params=(8.2, 0.2)):
    pr = np.asarray(params, dtype=np.float64)
    d = ctypes.c_double()
    a = ctypes.c_double()
    lib().or_cbpr2_coeffs(_p(pr), ctypes.byref(d), ctypes.byref(a))
    return d.value, a.value


def rhs_ones(N: int) -> np.ndarray:
    """b = A*1 as every reference driver builds it (test_poisson_mf.f90:39-40)."""
    return stvec(np.ones(N * N), N)


@dataclass
class SolveResult:
    x: np.ndarray
    final_err: np.ndarray
    v_err: np.ndarray
    n_out: int
    cycles_out: int          # restart_out (MGS-R) / stages_out (HH)
    hist_res: np.ndarray     # true relative residual after each cycle
    hist_ferr: np.ndarray    # (cycles, m) final_err of every step of every cycle
    cut: bool = False
    step_times: np.ndarray | None = field(default=None)

    @property
    def iterations(self) -> int:
        """(stages-1)*m + n_out, as test_poisson_mf.f90:47 prints it."""
        return (self.cycles_out - 1) * self.hist_ferr.shape[1] + self.n_out


def _solve(fn, b, N, m, tol, prec, params, degree, variant, max_cycles, step_limit, threads):
    set_threads(threads)
    n = N * N
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1)
    x = np.zeros(n)
    fe = np.zeros(m)
    ve = np.zeros(m + 1)
    n_out = ctypes.c_int()
    cyc_out = ctypes.c_int()
    ncyc = ctypes.c_int(0)
    hr = np.zeros(max_cycles)
    hf = np.zeros(max_cycles * m)
    pr = np.asarray(params if params is not None else (0.0, 0.0), dtype=np.float64)
    st = np.zeros(step_limit) if step_limit > 0 else None
    cut = fn(_p(b), N, m, tol, prec, _p(pr), degree, variant, max_cycles, _p(x), _p(fe),
             _p(ve), ctypes.byref(n_out), ctypes.byref(cyc_out), _p(hr), _p(hf),
             ctypes.byref(ncyc), step_limit, _p(st))
    set_threads(1)
    nc = ncyc.value
    return SolveResult(x=x, final_err=fe, v_err=ve, n_out=n_out.value, cycles_out=cyc_out.value,
                       hist_res=hr[:nc].copy(), hist_ferr=hf[: nc * m].reshape(nc, m).copy(),
                       cut=bool(cut), step_times=st)


def gmres_mgsr(b, N, m, tol=1e-15, prec=PREC_IDENTITY, params=(8.2, 0.2), degree=8,
               variant=MGSR_MF, max_cycles=1000, step_limit=0, threads=1) -> SolveResult:
    """gmres_mgsr_mf (variant MGSR_MF) / gmres_mgsr_omp (MGSR_OMP), gmres_mgsr.f90."""
    return _solve(lib().or_gmres_mgsr, b, N, m, tol, prec, params, degree, variant,
                  max_cycles, step_limit, threads)


def gmres_hh(b, N, m, tol=1e-15, prec=PREC_IDENTITY, params=(8.2, 0.2), degree=8,
             midcycle_exit=0, max_cycles=1000, step_limit=0, threads=1) -> SolveResult:
    """gmres_hh_omp (midcycle_exit=0, prec must be identity) / gmres_hh_prec_omp (=1)."""
    return _solve(lib().or_gmres_hh, b, N, m, tol, prec, params, degree, midcycle_exit,
                  max_cycles, step_limit, threads)


def _short_recurrence(fn, b, N, tol, max_iter, prec, params, degree):
    b = np.ascontiguousarray(b, dtype=np.float64).reshape(-1)
    x = np.zeros(N * N)
    it = ctypes.c_int(max_iter)
    res = ctypes.c_double()
    hist = np.zeros(max_iter)
    pr = np.asarray(params, dtype=np.float64)
    fn(_p(b), N, tol, ctypes.byref(it), ctypes.byref(res), prec, _p(pr), degree, _p(x), _p(hist))
    k = int(np.count_nonzero(hist))
    return x, it.value, res.value, hist[:k].copy()


def pcg(b, N, tol=1e-9, max_iter=1000, prec=PREC_IDENTITY, params=(8.2, 0.2), degree=8):
    """pcg_omp (src/cg.f90:154-234): returns (x, iter, res, per-iteration res)."""
    return _short_recurrence(lib().or_pcg, b, N, tol, max_iter, prec, params, degree)


def pbicgstab(b, N, tol=1e-9, max_iter=1000, prec=PREC_IDENTITY, params=(8.2, 0.2), degree=8):
    """pbicgstab_omp (src/bicgstab.f90:91-182): returns (x, iters, res, per-iteration res)."""
    return _short_recurrence(lib().or_pbicgstab, b, N, tol, max_iter, prec, params, degree)
