#!/usr/bin/env python3
"""A/B launch-policy variants of the GMRES(m) cycle in ONE process, interleaved
rounds (cdna_hip_programming.md 5.4 rule 24).  Each measurement is one full
restart cycle from x0 = 0 (identical work every time).

  python tools/tune.py --grid 4096 --m 95 --rounds 3 --variants nt=0,nt=1 nt=1:pj=1024 ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = {"nt": 0, "pj": 1, "st": 2, "rev": 3, "blk": 4, "unr": 5, "cf": 6, "res": 8, "rr2": 9, "lds": 12, "wo": 13}
DEFAULTS = {0: -1, 1: 0, 2: 0, 3: 0, 4: 0, 5: 0, 6: 1, 8: -1, 9: 0, 12: 1, 13: -1}


def parse_variant(s: str) -> dict:
    out = {}
    if s in ("base", "default"):
        return out
    for kv in s.split(":"):
        k, v = kv.split("=")
        out[KEYS[k]] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--m", type=int, default=95)
    ap.add_argument("--prec", default="identity")
    ap.add_argument("--degree", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", nargs="+", default=["base", "nt=1"])
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import gmres_amd as ga

    ctx = ga.Context(a.grid, a.m)
    ctx.set_precond(a.prec, (8.2, 0.2), a.degree)
    ctx.set_rhs_ones()
    ga.gmres_mgsr(ctx, 1e-15, max_cycles=1, want_verr=False)  # warm
    res = {v: {"wall_ms": [], "proj_us": [], "resid": None} for v in a.variants}
    for r in range(a.rounds):
        for v in a.variants:
            for k in KEYS.values():
                ctx.tune(k, DEFAULTS[k])
            for k, val in parse_variant(v).items():
                ctx.tune(k, val)
            ctx.sync()
            t0 = time.perf_counter()
            out = ga.gmres_mgsr(ctx, 1e-15, max_cycles=1, want_verr=False)
            ctx.sync()
            res[v]["wall_ms"].append((time.perf_counter() - t0) * 1e3)
            res[v]["resid"] = ctx.true_residual()
            ctx.profile(True)
            ctx.profile_reset()
            ga.gmres_mgsr(ctx, 1e-15, max_cycles=1, want_verr=False)
            p = ctx.profile_read()
            ctx.profile(False)
            res[v]["proj_us"].append(p["proj"][0] * 1e3 / max(p["proj"][1], 1) if p["proj"][1] else p["res"][0] * 1e3 / max(p["res"][1], 1))
            res[v]["breakdown_ms"] = {k: round(x[0], 3) for k, x in p.items()}
            print(json.dumps({"round": r, "variant": v, "wall_ms": round(res[v]["wall_ms"][-1], 2),
                              "proj_us": round(res[v]["proj_us"][-1], 2), "resid": res[v]["resid"]}), flush=True)
    summary = {v: {"wall_ms_min": round(min(d["wall_ms"]), 2), "wall_ms_med": round(sorted(d["wall_ms"])[len(d["wall_ms"]) // 2], 2),
                   "proj_us_min": round(min(d["proj_us"]), 2), "resid": d["resid"], "breakdown_ms": d["breakdown_ms"]}
               for v, d in res.items()}
    print(json.dumps({"grid": a.grid, "m": a.m, "prec": a.prec, "summary": summary}, indent=1))
    if a.out:
        json.dump({"grid": a.grid, "m": a.m, "prec": a.prec, "summary": summary, "raw": res}, open(a.out, "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
