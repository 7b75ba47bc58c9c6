"""final_err(94) / final_err(95) of cycle 1 at the split grids (one context, 1 GPU), MGS-R and
Householder: the reference is re-run with a tol between them (tests/golden/make_ref_fixtures.py
SPLIT_FE) so that it stops after exactly one full cycle and prints final_err(1:95) and x."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gmres_amd as ga  # noqa: E402

out = {}
for N in (1448, 2048, 2896):
    for method in ("mgsr", "hh"):
        with ga.Context(N, 95) as c:
            c.set_rhs_ones()
            if method == "mgsr":
                r = ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False, want_hist=True)
            else:
                r = ga.gmres_hh(c, 1e-15, precondition=False, max_cycles=1, want_verr=False, want_hist=True)
            out[f"{method}_{N}"] = {"fe94": float(r.final_err[93]), "fe95": float(r.final_err[94]),
                                    "n_out": int(r.n_out)}
        print(method, N, out[f"{method}_{N}"], flush=True)
print(json.dumps(out))
