#!/usr/bin/env python3
"""How far do slab solves (2 / 3 ranks through the device exchange on one GPU)
drift from the single-context solve, per residual tier?  The cases of
tests/test_gpu_xgmi.py::test_slabs_match_single_context; one JSON line per
case with the max relative deviation of the per-cycle true residual where the
reference residual is > 1e-6, in (1e-10, 1e-6], and <= 1e-10 -- the numbers the
tests' tolerances are set from.

  python tools/multirank_dev.py [--resident]

--resident forces the resident launches with the in-launch exchange
(GK_TUNE_RES = 1), the cases of test_resident_step_over_device_exchange.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["GPU_MAX_HW_QUEUES"] = "16"  # as tests/conftest.py: one queue per rank's stream


def main() -> None:
    import test_gpu_xgmi as T

    resident = "--resident" in sys.argv[1:]

    N, m, cyc = 66, 16, 6
    for method, prec, degree in [("mgsr", "identity", 1), ("mgsr", "cbpr2", 1), ("mgsr", "cheb", 4),
                                 ("hh", "identity", 1), ("hh", "cbpr2", 1)]:
        for nranks in ((2,) if resident else (2, 3)):
            ref = T._single(N, m, method, prec, degree, cyc)
            g, ctxs = T._local_group(N, m, nranks)

            def work(r):
                c = ctxs[r]
                if resident:
                    c.tune(8, 1)  # GK_TUNE_RES
                    c.tune(11, 5000)  # exchange deadline, ms
                c.set_precond(prec, (8.2, 0.2), degree)
                c.set_rhs_ones()
                return T._solve(c, method, prec, cyc)

            res = T._run_threads(nranks, work)
            T._close(g, ctxs)
            k = min(len(ref.hist_res), len(res[0].hist_res))
            h, rr = res[0].hist_res[:k], ref.hist_res[:k]
            dev = np.abs(h - rr) / rr
            tiers = {"gt_1e-6": rr > 1e-6, "1e-10_1e-6": (rr <= 1e-6) & (rr > 1e-10), "le_1e-10": rr <= 1e-10}
            out = {"resident": resident, "method": method, "prec": prec, "nranks": nranks, "cycles": int(k),
                   "last_residual": float(rr[-1])}
            for name, sel in tiers.items():
                out[name] = float(dev[sel].max()) if sel.any() else None
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
