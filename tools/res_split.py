#!/usr/bin/env python3
"""Where does a resident launch spend its time?  One warm cycle, then one cycle
with the in-kernel clock split on (gk_profile_res_split): per projection
(MGS-R) or reflection (Householder UP / DOWN chains), the mean over workgroups
of the time streaming the pass vs waiting in the in-launch all-gather.

  python tools/res_split.py [--grid 4096] [--m 95] [--method mgsr|hh|both]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--m", type=int, default=95)
    ap.add_argument("--method", default="both", choices=["mgsr", "hh", "both"])
    a = ap.parse_args()
    import gmres_amd as ga

    m = a.m
    with ga.Context(a.grid, m) as c:
        c.set_rhs_ones()
        for method in (["mgsr", "hh"] if a.method == "both" else [a.method]):
            run = (lambda: ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)) if method == "mgsr" else \
                (lambda: ga.gmres_hh(c, 1e-15, max_cycles=1, want_verr=False))
            c.zero_x()
            run()
            c.zero_x()
            c.res_split(1)
            run()
            c.sync()
            if method == "mgsr":
                kinds = [(0, "mgs_step", m * (m + 1))]  # 2j projections per step j
            else:
                # UP: j reflections per step; DOWN: j per step + the x update (m) + a pre-dot pass each
                kinds = [(1, "hh_up", m * (m + 1) // 2), (2, "hh_down", m * (m + 1) // 2 + m)]
            for which, name, nproj in kinds:
                r = c.res_split(-1, which)
                out = {"grid": a.grid, "m": m, "launch": name, "launches": r["launches"],
                       "pass_ms": round(r["pass_ms"], 3), "wait_ms": round(r["wait_ms"], 3),
                       "total_ms": round(r["total_ms"], 3),
                       "per_unit_us": {"pass": round(r["pass_ms"] * 1e3 / nproj, 3),
                                       "wait": round(r["wait_ms"] * 1e3 / nproj, 3),
                                       "total": round(r["total_ms"] * 1e3 / nproj, 3)},
                       "units": nproj}
                pw, ww = c.res_split_wg(which)
                if len(pw):  # arrival skew: per-workgroup pass time, and by XCD (blockIdx % 8)
                    per = pw * 1e3 / nproj
                    out["wg_pass_us"] = {"min": round(float(per.min()), 3), "median": round(float(np.median(per)), 3),
                                         "max": round(float(per.max()), 3)}
                    out["xcd_pass_us"] = [round(float(per[k::8].mean()), 3) for k in range(min(8, len(per)))]
                print(json.dumps(out), flush=True)
            c.res_split(0)


if __name__ == "__main__":
    main()
