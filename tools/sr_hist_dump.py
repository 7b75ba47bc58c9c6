"""Dump the fused short-recurrence residual histories (gk_sr_*) of the cases the
reference's truncation fixtures cover, for calibrating the per-iteration bands
of tests/test_gpu_sr.py / test_gpu_solver.py offline.  GPU; prints one JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gmres_amd as ga  # noqa: E402

out = {}
for solver in ("pbicgstab", "pcg"):
    for prec in ("identity", "cbpr2"):
        for N, K, tol in ((128, 5000, 1e-9), (256, 5000, 1e-9), (4096, 50, 1e-9)):
            with ga.Context(N, 8) as c:
                c.set_precond(prec, (8.2, 0.2), 1)
                c.set_rhs_ones()
                if N == 4096:
                    s = ga.SrSolve(c, solver, tol, K)
                    s.iterate(K)
                    ex, _, _ = s.status()
                    h = s.history(ex)
                else:
                    _, _, _, h = getattr(ga, solver)(c, tol, K, want_hist=True)
            out[f"{solver}_{prec}_{N}"] = [float(v) for v in h]
print(json.dumps(out))
