"""Generate tests/golden/reference_runs.json + reference_x.npz by running the
REFERENCE itself (oracle/_ref/ref_driver: the reference's own Fortran solver
modules compiled from /root/reference/src, see oracle/Makefile.ref).

Build container only (needs the compiled reference).  The fixtures are data:
per-cycle true residuals, final_err(1:n_out), v_err, iteration counts, x (full
at N <= 64).  Run:  python tests/golden/make_ref_fixtures.py [--quick]
                    python tests/golden/make_ref_fixtures.py --only KEY[,KEY...]
(--only re-runs the named cases and merges them into the existing files.)
"""
from __future__ import annotations

import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import refrun  # noqa: E402

# (key, solver, N, m, prec, threads, max_cycles)
SMALL = [
    ("mgsr_mf_identity_32_m10", "mgsr_mf", 32, 10, "identity", 1, 0),
    ("mgsr_mf_identity_32_m30", "mgsr_mf", 32, 30, "identity", 1, 0),
    ("mgsr_mf_identity_64_m20", "mgsr_mf", 64, 20, "identity", 1, 0),
    ("mgsr_mf_identity_128_m30", "mgsr_mf", 128, 30, "identity", 1, 0),
    ("mgsr_omp_identity_128_m30", "mgsr_omp", 128, 30, "identity", 1, 0),
    ("mgsr_mf_cbpr2_64_m20", "mgsr_mf", 64, 20, "cbpr2", 1, 0),
    ("mgsr_omp_cbpr2_32_m10", "mgsr_omp", 32, 10, "cbpr2", 1, 0),
    ("mgsr_omp_cbpr2_64_m20", "mgsr_omp", 64, 20, "cbpr2", 1, 0),
    ("mgsr_omp_cbpr2_128_m30", "mgsr_omp", 128, 30, "cbpr2", 1, 0),
    ("hh_omp_identity_32_m10", "hh_omp", 32, 10, "identity", 1, 0),
    ("hh_omp_identity_64_m20", "hh_omp", 64, 20, "identity", 1, 0),
    ("hh_omp_identity_128_m30", "hh_omp", 128, 30, "identity", 1, 0),
    ("hh_prec_omp_cbpr2_32_m10", "hh_prec_omp", 32, 10, "cbpr2", 1, 0),
    ("hh_prec_omp_cbpr2_64_m20", "hh_prec_omp", 64, 20, "cbpr2", 1, 0),
    ("hh_prec_omp_cbpr2_128_m30", "hh_prec_omp", 128, 30, "cbpr2", 1, 0),
    ("pcg_omp_identity_48", "pcg_omp", 48, 5000, "identity", 1, 0),
    ("pcg_omp_cbpr2_48", "pcg_omp", 48, 5000, "cbpr2", 1, 0),
    ("pbicgstab_omp_identity_48", "pbicgstab_omp", 48, 5000, "identity", 1, 0),
    ("pbicgstab_omp_cbpr2_48", "pbicgstab_omp", 48, 5000, "cbpr2", 1, 0),
    # capped serial histories at config-2 size (SURVEY 8c known answers)
    ("mgsr_mf_identity_1024_m95_3cyc", "mgsr_mf", 1024, 95, "identity", 1, 3),
    ("mgsr_mf_cbpr2_1024_m95_3cyc", "mgsr_mf", 1024, 95, "cbpr2", 1, 3),
]
THREADED = [
    ("mgsr_omp_identity_128_m30_t8", "mgsr_omp", 128, 30, "identity", 8, 0),
    ("hh_omp_identity_128_m30_t8", "hh_omp", 128, 30, "identity", 8, 0),
    ("hh_omp_identity_1024_m95_3cyc_t8", "hh_omp", 1024, 95, "identity", 8, 3),
    ("mgsr_omp_identity_1024_m95_3cyc_t8", "mgsr_omp", 1024, 95, "identity", 8, 3),
    # full-size configs (1 cycle each): 1, 3 (cbpr2 reference leg), 5
    ("mgsr_omp_identity_4096_m95_1cyc_t8", "mgsr_omp", 4096, 95, "identity", 8, 1),
    ("mgsr_omp_cbpr2_4096_m95_1cyc_t8", "mgsr_omp", 4096, 95, "cbpr2", 8, 1),
    ("hh_omp_identity_4096_m95_1cyc_t8", "hh_omp", 4096, 95, "identity", 8, 1),
    # residual HISTORIES beyond cycle 1 (round 4): the two cycles the bench legs time at
    # 4096^2, and twelve cycles at config-2 size
    ("mgsr_omp_identity_4096_m95_2cyc_t8", "mgsr_omp", 4096, 95, "identity", 8, 2),
    ("mgsr_omp_cbpr2_4096_m95_2cyc_t8", "mgsr_omp", 4096, 95, "cbpr2", 8, 2),
    ("hh_omp_identity_4096_m95_2cyc_t8", "hh_omp", 4096, 95, "identity", 8, 2),
    ("mgsr_omp_identity_1024_m95_12cyc_t8", "mgsr_omp", 1024, 95, "identity", 8, 12),
    ("mgsr_omp_cbpr2_1024_m95_12cyc_t8", "mgsr_omp", 1024, 95, "cbpr2", 8, 12),
    ("hh_omp_identity_1024_m95_12cyc_t8", "hh_omp", 1024, 95, "identity", 8, 12),
    # round 5: the grids whose per-workgroup load stands for the 2 / 4 / 8-GPU splits
    # (tests/test_gpu_splits.py), cycle 1 of the reference itself
    ("mgsr_omp_identity_1448_m95_1cyc_t8", "mgsr_omp", 1448, 95, "identity", 8, 1),
    ("mgsr_omp_identity_2048_m95_1cyc_t8", "mgsr_omp", 2048, 95, "identity", 8, 1),
    ("mgsr_omp_identity_2896_m95_1cyc_t8", "mgsr_omp", 2896, 95, "identity", 8, 1),
    ("hh_omp_identity_1448_m95_1cyc_t8", "hh_omp", 1448, 95, "identity", 8, 1),
    ("hh_omp_identity_2048_m95_1cyc_t8", "hh_omp", 2048, 95, "identity", 8, 1),
    ("hh_omp_identity_2896_m95_1cyc_t8", "hh_omp", 2896, 95, "identity", 8, 1),
]
# round 5: pcg_omp / pbicgstab_omp residual HISTORIES (src/cg.f90:154-234,
# src/bicgstab.f90:91-182).  The reference records no history, so it is taken
# by truncation: the solver run from x0 = 0 with max_iter = k returns the
# residual of iteration k (one serial process per k: pbicgstab_omp reads its
# dot accumulators uninitialised, so no two runs share a process).
KHIST = [
    ("pcg_omp_identity_128_hist", "pcg_omp", 128, "identity"),
    ("pcg_omp_cbpr2_128_hist", "pcg_omp", 128, "cbpr2"),
    ("pbicgstab_omp_identity_128_hist", "pbicgstab_omp", 128, "identity"),
    ("pbicgstab_omp_cbpr2_128_hist", "pbicgstab_omp", 128, "cbpr2"),
    ("pcg_omp_identity_256_hist", "pcg_omp", 256, "identity"),
    ("pcg_omp_cbpr2_256_hist", "pcg_omp", 256, "cbpr2"),
    ("pbicgstab_omp_identity_256_hist", "pbicgstab_omp", 256, "identity"),
    ("pbicgstab_omp_cbpr2_256_hist", "pbicgstab_omp", 256, "cbpr2"),
]

# round 6: (a) the same truncation histories for 50 iterations at the bench's
# 4096^2 (the fused device passes' full-size pin), and (b) BiCGSTAB's 256^2
# identity history at 8 threads beside the 1-thread one above: the spread of the
# reference against itself (reduction order only) sets the per-iteration band
# of tests/test_gpu_solver.py's BiCGSTAB history test.
# (key, solver, N, prec, iterations, threads)
KHIST_CAP = [
    ("pcg_omp_identity_4096_hist50", "pcg_omp", 4096, "identity", 50, 1),
    ("pcg_omp_cbpr2_4096_hist50", "pcg_omp", 4096, "cbpr2", 50, 1),
    ("pbicgstab_omp_identity_4096_hist50", "pbicgstab_omp", 4096, "identity", 50, 1),
    ("pbicgstab_omp_cbpr2_4096_hist50", "pbicgstab_omp", 4096, "cbpr2", 50, 1),
    ("pbicgstab_omp_identity_4096_hist50_t8", "pbicgstab_omp", 4096, "identity", 50, 8),
    ("pbicgstab_omp_cbpr2_4096_hist50_t8", "pbicgstab_omp", 4096, "cbpr2", 50, 8),
    ("pbicgstab_omp_identity_256_hist_t8", "pbicgstab_omp", 256, "identity", 0, 8),
    ("pbicgstab_omp_cbpr2_256_hist_t8", "pbicgstab_omp", 256, "cbpr2", 0, 8),
    ("pbicgstab_omp_identity_128_hist_t8", "pbicgstab_omp", 128, "identity", 0, 8),
    ("pbicgstab_omp_cbpr2_128_hist_t8", "pbicgstab_omp", 128, "cbpr2", 0, 8),
    ("pcg_omp_identity_256_hist_t8", "pcg_omp", 256, "identity", 0, 8),
]


# round 6: cycle 1 at the split grids IN FULL -- final_err(1:95) and x, which a run cut after
# one cycle never prints.  tol between the cycle's final_err(94) and final_err(95) (both
# ~0.00304 / ~0.00299 at these grids, tools/split_fe_dump.py) ends the solve normally at the
# end of cycle 1 (gmres_mgsr.f90:385-389 / 409-412; gmres_hh.f90's end-of-cycle test).
# x is kept as a sample: every X_STRIDE-th unknown.  (key, solver, N, threads, tol)
SPLIT_FE_TOL = 0.00301
X_STRIDE = 4099
SPLIT_FE = [(f"{s}_identity_{N}_m95_cyc1full_t8", s, N, 8, SPLIT_FE_TOL)
            for N in (1448, 2048, 2896) for s in ("mgsr_omp", "hh_omp")]


def record_split_fe(key, solver, N, threads, tol):
    t0 = time.time()
    r = refrun.run(solver, N, 95, "identity", threads=threads, want_x=True, env={"REF_TOL": repr(tol)})
    assert not r.cut and r.cycles_out == 1 and r.n_out == 95, (key, r.cycles_out, r.n_out)
    idx = np.arange(0, N * N, X_STRIDE)
    d = {"solver": solver, "N": N, "m": 95, "prec": "identity", "threads": r.threads, "tol": tol,
         "n_out": r.n_out, "cycles": r.cycles_out, "final_err": r.final_err.tolist(), "x_err": list(r.x_err),
         "final_res": r.final_res, "x_stride": X_STRIDE, "x_sample": r.x[idx].tolist(),
         "note": "one full cycle (tol between final_err(94) and final_err(95)); x_sample = x[::x_stride]",
         "wall_s": round(time.time() - t0, 2)}
    print(f"{key}: {time.time() - t0:.1f} s", flush=True)
    return key, d


def record_khist_cap(key, solver, N, prec, K, threads):
    """Truncation history of iterations 1..K (K = 0: to convergence) with
    `threads` OpenMP threads per run (runs in parallel, 8 cores in all)."""
    t0 = time.time()
    if K == 0:
        K = refrun.run(solver, N, 5000, prec, threads=threads).krylov[0]
    pts = hist_points(K)
    par = max(1, 8 // threads)
    with ThreadPoolExecutor(par) as ex:
        hist = list(ex.map(lambda k: refrun.run(solver, N, k, prec, threads=threads).krylov[1], pts))
    d = {"solver": solver, "N": N, "prec": prec, "threads": threads, "tol": 1e-9, "hist_iter": pts,
         "hist_res": hist,
         "note": "hist_res[i] = the reference's residual after hist_iter[i] iterations (run truncated there)",
         "wall_s": round(time.time() - t0, 2)}
    print(f"{key}: {K} history points, {time.time() - t0:.1f} s", flush=True)
    return key, d


def hist_points(K: int) -> list[int]:
    """Iterations of a truncation history: every one."""
    return list(range(1, K + 1))


def record_khist(key, solver, N, prec):
    t0 = time.time()
    full = refrun.run(solver, N, 5000, prec, threads=1)
    K, res = full.krylov
    pts = hist_points(K)
    with ThreadPoolExecutor(6) as ex:
        hist = list(ex.map(lambda k: refrun.run(solver, N, k, prec, threads=1).krylov[1], pts))
    d = {"solver": solver, "N": N, "m": 5000, "prec": prec, "threads": 1, "cut": False, "tol": 1e-9, "iterations": K,
         "res": res,
         "hist_iter": pts, "hist_res": hist, "x_err": list(full.x_err),
         "note": "hist_res[i] = the reference's residual after hist_iter[i] iterations (run truncated there)",
         "wall_s": round(time.time() - t0, 2)}
    print(f"{key}: {K} iterations, {len(pts)} history points, {time.time() - t0:.1f} s", flush=True)
    return key, d


def record(key, solver, N, m, prec, threads, max_cycles):
    t0 = time.time()
    r = refrun.run(solver, N, m, prec, threads=threads, max_cycles=max_cycles, want_x=N <= 64)
    d = {"solver": solver, "N": N, "m": m, "prec": prec, "threads": r.threads, "max_cycles": max_cycles,
         "cut": r.cut, "hist_res": r.hist_res.tolist(), "wall_s": round(time.time() - t0, 2)}
    if r.krylov is not None:
        d["iterations"], d["res"] = r.krylov
        d["x_err"] = list(r.x_err)
    elif not r.cut:
        d.update(iterations=r.iterations, cycles=r.cycles_out, n_out=r.n_out, final_err=r.final_err.tolist(),
                 v_err=r.v_err.tolist(), x_err=list(r.x_err), time_s=r.time)
    print(f"{key}: {time.time() - t0:.1f} s", flush=True)
    return key, d, r.x


def main() -> None:
    quick = "--quick" in sys.argv
    only = None
    if "--only" in sys.argv:
        only = set(sys.argv[sys.argv.index("--only") + 1].split(","))
        unknown = only - {c[0] for c in SMALL + THREADED + KHIST + KHIST_CAP + SPLIT_FE}
        if unknown:
            raise SystemExit(f"unknown cases {sorted(unknown)}")
    refrun.build()
    small = [c for c in SMALL if (not quick or c[2] <= 128) and (only is None or c[0] in only)]
    out, xs = {}, {}
    with ThreadPoolExecutor(6) as ex:
        for key, d, x in ex.map(lambda c: record(*c), small):
            out[key] = d
            if x is not None:
                xs[key] = x
    for c in THREADED:
        if (quick and c[2] > 128) or (only is not None and c[0] not in only):
            continue
        key, d, x = record(*c)
        out[key] = d
        if x is not None:
            xs[key] = x
    for c in KHIST:
        if (quick and c[2] > 128) or (only is not None and c[0] not in only):
            continue
        key, d = record_khist(*c)
        out[key] = d
    for c in KHIST_CAP:
        if (quick and c[2] > 128) or (only is not None and c[0] not in only):
            continue
        key, d = record_khist_cap(*c)
        out[key] = d
    for c in SPLIT_FE:
        if quick or (only is not None and c[0] not in only):
            continue
        key, d = record_split_fe(*c)
        out[key] = d
    meta = {"_source": "oracle/_ref/ref_driver: the reference's own src/*.f90 (AlexanderGSC/gmres) compiled "
                       "by oracle/Makefile.ref (amdflang 22, -O3 -fopenmp -funroll-loops; interfaces.f90 "
                       "with the one-line import fix), driven through the stencil_vector/precond seam by "
                       "oracle/ref_driver.f90; b = A*1, x0 = 0, tol 1e-15 (CG/BiCGSTAB 1e-9), params (8.2, 0.2)",
            "_generator": "tests/golden/make_ref_fixtures.py"}
    path = os.path.join(HERE, "reference_runs.json")
    merge = quick or only is not None
    old = json.load(open(path)) if os.path.exists(path) and merge else {}
    old.update(out)
    old.update(meta)
    json.dump(dict(sorted(old.items())), open(path, "w"), indent=1)
    xpath = os.path.join(HERE, "reference_x.npz")
    if merge and os.path.exists(xpath):
        with np.load(xpath) as f:
            xs = {**{k: f[k] for k in f.files}, **xs}
    np.savez_compressed(xpath, **xs)


if __name__ == "__main__":
    main()
