#!/usr/bin/env python3
"""Short fixed workload for rocprofv3 PMC passes: one GMRES(m) cycle with a
small m on the full-size grid.  Projection launches do the same work for
every j, so per-launch counters equal those of the m=95 bench."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=4096)
ap.add_argument("--m", type=int, default=8)
ap.add_argument("--prec", default="identity")
ap.add_argument("--nt", type=int, default=-1)
a = ap.parse_args()
import gmres_amd as ga

ctx = ga.Context(a.grid, a.m)
ctx.tune(0, a.nt)
ctx.set_precond(a.prec)
ctx.set_rhs_ones()
r = ga.gmres_mgsr(ctx, 1e-15, max_cycles=1, want_verr=False)
ctx.sync()
print("probe done", a.grid, a.m, r.n_out)
ctx.close()
