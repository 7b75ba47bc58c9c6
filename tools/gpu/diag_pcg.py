"""Diagnostic: pcg_omp with cbpr2 on the device vs the reference's truncation history."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import gmres_amd as ga  # noqa: E402

R = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_runs.json")))
for N in (64, 128, 192, 256):
    for m in (8, 30):
        with ga.Context(N, m) as ctx:
            ctx.set_precond("cbpr2", (8.2, 0.2), 4)
            ctx.set_rhs_ones()
            x, it, res, hist = ga.pcg(ctx, 1e-9, 5000, want_hist=True)
        key = f"pcg_omp_cbpr2_{N}_hist"
        ref = R.get(key)
        line = f"N={N} m={m}: {it} iterations res {res:.3e}; hist[:4] {np.asarray(hist[:4])}"
        if ref:
            line += f" ref {ref['iterations']} {np.asarray(ref['hist_res'][:4])}"
        print(line, flush=True)
