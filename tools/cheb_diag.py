#!/usr/bin/env python3
"""Where does a Chebyshev pass differ from the oracle?  For each (N, degree):
one preconditioner application on random input, compared element-wise with
the CPU oracle (the checker); prints the mismatch count and the row / column
ranges of the mismatches (grid coordinates: j = line, i = fast index).

  python tools/cheb_diag.py --grids 1024 4096 --degrees 1 8
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", type=int, nargs="+", default=[1024])
    ap.add_argument("--degrees", type=int, nargs="+", default=[8])
    a = ap.parse_args()
    import torch

    import gmres_amd.solver as S
    from oracle import oracle as orc  # the checker

    def report(tag, N, k, z, ref):
        bad = np.nonzero(z != ref)[0]
        out = {"path": tag, "N": N, "degree": k, "mismatches": int(bad.size)}
        if bad.size:
            j, i = bad // N, bad % N
            out.update({"rows": [int(j.min()), int(j.max())], "cols": [int(i.min()), int(i.max())],
                        "distinct_rows": int(np.unique(j).size), "distinct_cols": int(np.unique(i).size),
                        "max_rel_dev": float(np.abs(z - ref).max() / np.abs(ref).max()),
                        "rows_sample": np.unique(j)[:16].tolist(), "cols_sample": np.unique(i)[:16].tolist()})
        print(json.dumps(out), flush=True)

    import gmres_amd as ga
    from gmres_amd import _native as nat

    for N in a.grids:
        for k in a.degrees:
            # the ACC_NORM pass of the cycle start: V(:,1) = w / beta with w = M^-1 b
            w = orc.precond(orc.PREC_CHEB, orc.rhs_ones(N), N, params=(8.2, 0.2), degree=k)
            for rep in range(2):
                with ga.Context(N, 4) as c:
                    c.tune(8, 0)  # launch path: the cycle start is the same either way
                    c.set_precond("cheb", (8.2, 0.2), k)
                    c.set_rhs_ones()
                    beta = c.mgs_cycle_start()
                    nat.check(nat.hip().gk_vec_lincomb(c.handle, 0, 0, 2, 0, 0, 0.0, 0.0), "gk_vec_lincomb")
                    v1 = c.get_x()
                report(f"norm_epilogue_rep{rep}", N, k, v1 * beta, w)
                print(json.dumps({"beta": beta, "ref_beta": float(np.sqrt(np.sum(w * w)))}))

            r = np.random.default_rng(N + k).standard_normal(N * N)
            rd = torch.from_numpy(r).to("cuda")
            zd = torch.empty_like(rd)
            scratch = torch.empty(3 * N * N, dtype=torch.float64, device="cuda")
            S.precond_apply(rd, zd, N, kind="cheb", params=(8.2, 0.2), degree=k, scratch=scratch)
            torch.cuda.synchronize()
            z = zd.cpu().numpy()
            ref = orc.precond(orc.PREC_CHEB, r, N, params=(8.2, 0.2), degree=k)
            bad = np.nonzero(z != ref)[0]
            out = {"N": N, "degree": k, "mismatches": int(bad.size)}
            if bad.size:
                j, i = bad // N, bad % N
                out.update({"rows": [int(j.min()), int(j.max())], "cols": [int(i.min()), int(i.max())],
                            "distinct_rows": int(np.unique(j).size), "distinct_cols": int(np.unique(i).size),
                            "first": [int(j[0]), int(i[0])], "max_abs_dev": float(np.abs(z - ref).max()),
                            "rows_sample": np.unique(j)[:12].tolist(), "cols_sample": np.unique(i)[:12].tolist()})
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
