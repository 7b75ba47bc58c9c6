#!/usr/bin/env python3
"""How many workgroups should a resident MGS-R step use on a small slab?
GK_TUNE_RES_SHARE = s gives the launch CUs / s workgroups (more data per
workgroup, fewer producers and readers per all-gather).  Times whole cycles of
one solve per setting, interleaved over rounds.

  python tools/tune_res_share.py [--grid 1024] [--m 95] [--shares 1,2,4] [--rounds 2] [--cycles 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--m", type=int, default=95)
    ap.add_argument("--shares", default="1,2,4")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--cycles", type=int, default=5)
    a = ap.parse_args()
    import gmres_amd as ga

    out = {}
    with ga.Context(a.grid, a.m) as c:
        c.set_rhs_ones()
        for r in range(a.rounds):
            for s in [int(x) for x in a.shares.split(",")]:
                c.tune(8, 1)   # GK_TUNE_RES on (share > 1 would switch auto mode off)
                c.tune(10, s)  # GK_TUNE_RES_SHARE
                c.zero_x()
                ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)  # warm
                c.zero_x()
                c.sync()
                t0 = time.perf_counter()
                res = ga.gmres_mgsr(c, 1e-15, max_cycles=a.cycles, want_verr=False, want_hist=True)
                c.sync()
                dt = time.perf_counter() - t0
                it = (res.n_cycles - 1) * a.m + res.n_out
                row = {"grid": a.grid, "share": s, "round": r, "it_s": round(it / dt, 2),
                       "per_projection_us": round(dt / (res.n_cycles * a.m * (a.m + 1)) * 1e6, 3),
                       "resid": float(res.hist_res[-1]) if len(res.hist_res) else None}
                out.setdefault(s, []).append(row["it_s"])
                print(json.dumps(row), flush=True)
    print(json.dumps({"summary": {str(k): max(v) for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
