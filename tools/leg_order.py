#!/usr/bin/env python3
"""Why do bench.py's config legs run slower per cycle than the same config as
the headline?  Runs fresh-context legs (1 warmup cycle, K timed cycles, no
profiling) in the order given, in ONE process, and prints ms per cycle per leg
plus the host-side split: the wall time of the K cycles minus the device time
of the step launches is the host / gap time.

  python tools/leg_order.py --legs cheb identity cheb --torch-sync
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", nargs="+", default=["cheb", "identity", "cheb"])
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--cycles", type=int, default=2)
    ap.add_argument("--torch-sync", action="store_true", help="torch.cuda.synchronize() before the first leg")
    ap.add_argument("--pre-grid", type=int, default=0,
                    help="before the legs: one identity cycle on a context of this grid, then close it")
    ap.add_argument("--prof", type=int, default=0, help="HIP events every S-th step in the timed cycles (bench: 16)")
    ap.add_argument("--hist-warm", action="store_true", help="warmup cycle with the per-cycle true residual")
    ap.add_argument("--method", default="mgsr", choices=["mgsr", "hh"])
    ap.add_argument("--keep-x", action="store_true", help="timed solve leaves x in HBM (no final download)")
    a = ap.parse_args()
    import torch

    import gmres_amd as ga

    if a.torch_sync:
        torch.cuda.synchronize(0)
    if a.pre_grid:
        with ga.Context(a.pre_grid, 95) as c:
            c.set_rhs_ones()
            ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)
            c.sync()
    for i, prec in enumerate(a.legs):
        deg = 8 if prec == "cheb" else 1
        with ga.Context(a.grid, 95) as c:
            c.set_precond(prec, (8.2, 0.2), deg)
            c.set_rhs_ones()

            def run(k, hist=False, want_x=True):
                if a.method == "mgsr":
                    return ga.gmres_mgsr(c, 1e-15, max_cycles=k, want_verr=False, want_hist=hist, want_x=want_x)
                return ga.gmres_hh(c, 1e-15, precondition=prec != "identity", max_cycles=k, want_verr=False,
                                   want_hist=hist, want_x=want_x)

            run(1, a.hist_warm)
            if a.prof:
                c.profile(a.prof)
                c.profile_reset()
            c.sync()
            t0 = time.perf_counter()
            r = run(a.cycles, want_x=not a.keep_x)
            c.sync()
            t1 = time.perf_counter()
        iters = (r.n_cycles - 1) * 95 + r.n_out
        print(json.dumps({"leg": i, "prec": prec, "grid": a.grid, "method": a.method, "prof": a.prof,
                          "hist_warm": a.hist_warm, "pre_grid": a.pre_grid, "keep_x": a.keep_x, "ms_per_cycle": round((t1 - t0) / r.n_cycles * 1e3, 3),
                          "it_s": round(iters / (t1 - t0), 3)}), flush=True)


if __name__ == "__main__":
    main()
