"""Run the REFERENCE itself (oracle/_ref/ref_driver: AlexanderGSC/gmres's own
Fortran solver modules, compiled from /root/reference/src by
oracle/Makefile.ref, driven through their operator seam by
oracle/ref_driver.f90).

TEST INFRASTRUCTURE ONLY: used to make the golden fixtures
(tests/golden/make_ref_fixtures.py), by tests/ as a checker, and by bench.py's
cpu_baseline leg (kind "reference").  Never imported by gmres_amd/.

/root/reference exists only in the build container: build() is a no-op
elsewhere and the prebuilt oracle/_ref/ref_driver travels with the tree.
"""
from __future__ import annotations

import os
import subprocess
import tempfile
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")
EXE = os.path.join(REF_DIR, "ref_driver")
REFERENCE = os.environ.get("GMRES_REFERENCE", "/root/reference")

SOLVERS = ("mgsr_mf", "mgsr_omp", "hh_omp", "hh_prec_omp", "pcg_omp", "pbicgstab_omp")


def build() -> str | None:
    """Compile oracle/_ref/ref_driver from the reference sources (build
    container only; returns None where /root/reference is absent)."""
    if not os.path.isdir(os.path.join(REFERENCE, "src")):
        return EXE if os.path.exists(EXE) else None
    subprocess.run(["make", "-s", "-C", HERE, "-f", "Makefile.ref", f"REF={REFERENCE}"], check=True)
    return EXE


def available() -> bool:
    return os.path.exists(EXE) and os.access(EXE, os.X_OK)


@dataclass
class RefRun:
    solver: str
    N: int
    m: int
    prec: str
    threads: int
    cut: bool
    cycle_res: list[float] = field(default_factory=list)      # true rel. residual at the start of cycle k (k>=2)
    cycle_t: list[float] = field(default_factory=list)        # omp_get_wtime stamp (s, logging excluded)
    step_t: dict[int, float] = field(default_factory=dict)    # stamp at the start of Arnoldi step j of cycle 1
    time: float | None = None
    n_out: int | None = None
    cycles_out: int | None = None
    final_res: float | None = None
    final_err: np.ndarray | None = None
    v_err: np.ndarray | None = None
    x_err: tuple[float, float] | None = None                  # ||x-1||_2, ||x-1||_inf
    x: np.ndarray | None = None
    krylov: tuple[int, float] | None = None                   # (iterations, residual) of pcg/pbicgstab

    @property
    def hist_res(self) -> np.ndarray:
        """True relative residual after each completed cycle (the oracle's
        hist_res convention): cycle starts 2.. then the final x."""
        h = list(self.cycle_res)
        if not self.cut and self.final_res is not None:
            h.append(self.final_res)
        return np.array(h)

    @property
    def iterations(self) -> int:
        return (self.cycles_out - 1) * self.m + self.n_out


def run(solver: str, N: int, m: int, prec: str = "identity", threads: int = 1, max_cycles: int = 0,
        step_limit: int = 0, want_x: bool = False, timeout: float | None = None, env: dict | None = None) -> RefRun:
    if solver not in SOLVERS:
        raise ValueError(solver)
    if not available():
        raise FileNotFoundError(f"{EXE} not built (oracle/refrun.build() in the build container)")
    e = dict(os.environ)
    e.update({"OMP_NUM_THREADS": str(threads), "OMP_DYNAMIC": "false"})
    if env:
        e.update(env)
    with tempfile.TemporaryDirectory() as td:
        xf = os.path.join(td, "x.bin")
        cmd = [EXE, solver, str(N), str(m), prec, str(max_cycles), str(step_limit)] + ([xf] if want_x else [])
        p = subprocess.run(cmd, capture_output=True, text=True, env=e, timeout=timeout)
        if p.returncode != 0:
            raise RuntimeError(f"ref_driver failed ({p.returncode}): {p.stderr[-2000:]}")
        r = RefRun(solver=solver, N=N, m=m, prec=prec, threads=threads, cut=False)
        for line in p.stdout.splitlines():
            t = line.split()
            if not t:
                continue
            k = t[0]
            if k == "CYC":
                if int(t[1]) >= 2:
                    r.cycle_res.append(float(t[2]))
                r.cycle_t.append(float(t[3]))
            elif k == "STEP":
                r.step_t[int(t[1])] = float(t[2])
            elif k == "CUT":
                r.cut = True
            elif k == "RUN":
                r.threads = int(t[-1])
            elif k == "TIME":
                r.time = float(t[1])
            elif k == "OUT":
                r.n_out, r.cycles_out = int(t[1]), int(t[2])
            elif k == "FINALRES":
                r.final_res = float(t[1])
            elif k == "FERR":
                r.final_err = np.array([float(v) for v in t[2:]])
                assert r.final_err.size == int(t[1])
            elif k == "VERR":
                r.v_err = np.array([float(v) for v in t[2:]])
            elif k == "XERR":
                r.x_err = (float(t[1]), float(t[2]))
            elif k == "KRYLOV":
                # a truncated pbicgstab_omp run returns max_iter from an uninitialised
                # local (src/bicgstab.f90:182): the I8 field then prints as stars
                r.krylov = (int(t[1]) if t[1].lstrip("-").isdigit() else -1, float(t[2]))
        if want_x and not r.cut:
            r.x = np.fromfile(xf, dtype=np.float64)
    return r
