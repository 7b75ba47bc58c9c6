#!/usr/bin/env python3
"""Per-solve overhead of a GMRES(m) solve on one GPU: wall time of solves of
K = 1, 2, 4, 8 restart cycles (from x0 = 0, fresh solve each), least-squares
t(K) = a + b K.  `a` is what a short timed leg (bench.py config legs) pays on
top of its cycles; `b` the cycle time.  One JSON line per grid.

  python tools/solve_overhead.py --grid 1024 [--prof-every 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--m", type=int, default=95)
    ap.add_argument("--prof-every", type=int, default=0, help="HIP-event sampling as bench.py's legs (0 = off)")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import gmres_amd as ga

    with ga.Context(a.grid, a.m) as c:
        c.set_precond("identity", (8.2, 0.2), 1)
        c.set_rhs_ones()
        ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)  # warm
        if a.prof_every > 0:
            c.profile(a.prof_every)
        ks, ts = [], []
        for _ in range(a.reps):
            for k in (1, 2, 4, 8):
                c.sync()
                t0 = time.perf_counter()
                ga.gmres_mgsr(c, 1e-15, max_cycles=k, want_verr=False)
                c.sync()
                ks.append(k)
                ts.append(time.perf_counter() - t0)
    b, a0 = np.polyfit(ks, ts, 1)
    print(json.dumps({"grid": a.grid, "m": a.m, "prof_every": a.prof_every, "per_solve_s": round(float(a0), 5),
                      "per_cycle_s": round(float(b), 5), "samples": [[k, round(t, 5)] for k, t in zip(ks, ts)]}))


if __name__ == "__main__":
    main()
