"""Generate tests/golden fixtures.

1. reference_known_answers.json -- outputs of the REFERENCE Fortran itself
   (AlexanderGSC/gmres built with amdflang 22 -O3 -fopenmp in the survey
   container, instrumented through its operator seam), transcribed from
   SURVEY.md section 8(c) "Known answers".  The reference cannot be rebuilt
   unmodified in this image (amdflang rejects src/interfaces.f90:21, see
   DESIGN.md), so these recorded values are the pin; they are data, not code.
2. oracle_*.npz -- small input/output vectors produced by the CPU oracle
   (oracle/gmres_oracle.c) after it reproduced (1) bit for bit; used by the
   CPU tests and as GPU parity fixtures.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

KNOWN = {
    "_source": "SURVEY.md 8(c) Known answers: reference Fortran (amdflang 22, -O3 -fopenmp), b = A*1, x0 = 0, "
               "tol = 1e-15, params (8.2, 0.2)",
    "mgsr_identity_128_m30": {"solver": "gmres_mgsr_mf (== gmres_mgsr_omp at 1 thread)", "threads": 1,
                              "iterations": 3592, "cycles": 120, "final_err": 9.9297601797034485e-16,
                              "true_rel_residual": 2.0383e-15, "x_minus_1_l2": 1.845e-11},
    "mgsr_identity_128_m30_omp8": {"solver": "gmres_mgsr_omp", "threads": 8, "iterations": 3587, "cycles": 120,
                                   "final_err": 9.9702e-16},
    "mgsr_cbpr2_128_m30": {"solver": "gmres_mgsr_omp + cbpr2", "threads": 1, "iterations": 1056, "cycles": 36},
    "hh_cbpr2_128_m30": {"solver": "gmres_hh_prec_omp + cbpr2", "threads": 1, "iterations": 1056, "cycles": 36},
    "hh_identity_128_m30": {"solver": "gmres_hh_omp", "iterations": 3600, "cycles": 120, "v_err_approx": 9.5e-31},
    "mgsr_identity_1024_m95": {"solver": "gmres_mgsr_mf", "threads": 1,
                               "cycle_true_residual": [2.9910582138934039e-03, 1.1416421199862048e-03,
                                                       6.9436835052474476e-04]},
    "mgsr_cbpr2_1024_m95": {"solver": "gmres_mgsr_mf + cbpr2", "threads": 1,
                            "cycle_true_residual": [1.1116780150843835e-03, 4.1999818712023672e-04,
                                                    2.5349247477200900e-04]},
    "hh_identity_1024_m95": {"solver": "gmres_hh_omp", "threads": 8,
                             "cycle_true_residual": [2.9910582138931397e-03, 1.1416421200028050e-03,
                                                     6.9436835053583517e-04]},
    "mgsr_identity_4096_m95": {"solver": "gmres_mgsr_omp", "threads": 8, "cycle_true_residual": [2.9820e-03],
                               "digits": 5},
    "mgsr_cbpr2_4096_m95": {"solver": "gmres_mgsr_omp + cbpr2", "threads": 8, "cycle_true_residual": [1.1120e-03],
                            "digits": 5},
}


def main():
    with open(os.path.join(HERE, "reference_known_answers.json"), "w") as f:
        json.dump(KNOWN, f, indent=1)
    from oracle import oracle as orc

    orc.build()
    rng = np.random.default_rng(2026)
    out = {}
    for N in (8, 33, 64):
        x = rng.standard_normal(N * N)
        out[f"stvec_x_{N}"] = x
        out[f"stvec_y_{N}"] = orc.stvec(x, N)
        out[f"cbpr2_z_{N}"] = orc.precond(orc.PREC_CBPR2, x, N)
        out[f"cheb8_z_{N}"] = orc.precond(orc.PREC_CHEB, x, N, degree=8)
    np.savez_compressed(os.path.join(HERE, "oracle_operators.npz"), **out)
    sol = {}
    for N, m in ((32, 10), (32, 30)):
        b = orc.rhs_ones(N)
        for name, kw, fn in (("mgsr_id", dict(variant=orc.MGSR_OMP), orc.gmres_mgsr),
                             ("mgsr_cbpr2", dict(prec=orc.PREC_CBPR2, variant=orc.MGSR_OMP), orc.gmres_mgsr),
                             ("hh_id", dict(midcycle_exit=0), orc.gmres_hh),
                             ("hh_cbpr2", dict(prec=orc.PREC_CBPR2, midcycle_exit=1), orc.gmres_hh)):
            r = fn(b, N, m, **kw)
            key = f"{name}_{N}_m{m}"
            sol[key + "_x"] = r.x
            sol[key + "_hist_res"] = r.hist_res
            sol[key + "_iters"] = np.array([r.iterations])
            sol[key + "_final_err"] = r.final_err[: r.n_out]
    np.savez_compressed(os.path.join(HERE, "oracle_solves.npz"), **sol)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
