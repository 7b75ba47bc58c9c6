#!/usr/bin/env python3
"""Anatomy of the in-launch all-gathers of one resident launch
(gk_profile_res_trace).  For Arnoldi step j of a warm cycle, every workgroup
stamps (wall clock, 10 ns) when it published its partial of exchange p and when
it held the grid total.  Per exchange:

  last     = the latest publish (the straggler that every workgroup waits for)
  skew_g   = last - publish_g            (waiting for the slowest workgroup)
  prop_g   = seen_g - last               (granule propagation + poll + sweep)

Prints one JSON line per traced step: means / percentiles of skew and
propagation, the share of exchanges each XCD (blockIdx % 8) was last in, and
the spread of publish times per exchange.

  python tools/res_trace.py [--grid 4096] [--m 95] [--steps 16,48,80] [--tune 23=4]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def analyse(pub: np.ndarray, seen: np.ndarray) -> dict:
    """pub, seen: [workgroups, exchanges] in ms."""
    ok = (pub > 0).all(axis=0) & (seen > 0).all(axis=0)
    pub, seen = pub[:, ok], seen[:, ok]
    last = pub.max(axis=0)
    skew = (last[None, :] - pub) * 1e3
    prop = (seen - last[None, :]) * 1e3
    wait = (seen - pub) * 1e3
    G = pub.shape[0]
    who = pub.argmax(axis=0)
    xcd_last = np.bincount(who % 8, minlength=8) / max(1, len(who))
    # time from one exchange's latest publish to the next exchange's first publish:
    # the fastest workgroup's pass after the total was known
    gap = (pub[:, 1:].min(axis=0) - seen[:, :-1].max(axis=0)) * 1e3 if pub.shape[1] > 1 else np.zeros(1)
    pct = lambda v, q: round(float(np.percentile(v, q)), 3)  # noqa: E731
    # is lateness a property of the workgroup (static imbalance) or of the pass (noise)?
    late = (pub - np.median(pub, axis=0)[None, :]) * 1e3  # us behind the median publisher
    wg_late = late.mean(axis=1)
    h = late.shape[1] // 2
    persist = float(np.corrcoef(late[:, :h].mean(axis=1), late[:, h:].mean(axis=1))[0, 1]) if h >= 2 else 0.0
    # does being late at exchange p lengthen the next pass (seen_p -> publish_{p+1})?
    # (e.g. the L2 touch loads a late workgroup issued during a short wait still draining)
    follow = {}
    if pub.shape[1] > 1:
        nxt = (pub[:, 1:] - seen[:, :-1]) * 1e3
        lp = late[:, :-1]
        q90, q50 = np.percentile(lp, 90, axis=0), np.percentile(lp, 50, axis=0)
        follow = {"late10pct": round(float(nxt[lp >= q90[None, :]].mean()), 3),
                  "early50pct": round(float(nxt[lp <= q50[None, :]].mean()), 3),
                  "corr": round(float(np.corrcoef(lp.ravel(), nxt.ravel())[0, 1]), 3)}
    return {"workgroups": G, "exchanges": int(ok.sum()),
            "wait_us": {"mean": round(float(wait.mean()), 3), "p50": pct(wait, 50), "p90": pct(wait, 90)},
            "skew_us": {"mean": round(float(skew.mean()), 3), "p50": pct(skew, 50), "p90": pct(skew, 90),
                        "spread_per_exchange_mean": round(float(skew.max(axis=0).mean()), 3)},
            "prop_us": {"mean": round(float(prop.mean()), 3), "min": round(float(prop.min()), 3),
                        "p50": pct(prop, 50), "p90": pct(prop, 90), "max": round(float(prop.max()), 3)},
            "xcd_share_last": [round(float(v), 3) for v in xcd_last],
            "last_wg_most_often": int(np.bincount(who).argmax()),
            "wg_lateness_us": {"sd_of_wg_means": round(float(wg_late.std()), 3),
                               "sd_per_exchange": round(float(late.std(axis=0).mean()), 3),
                               "halves_correlation": round(persist, 3),
                               "by_xcd": [round(float(wg_late[k::8].mean()), 3) for k in range(min(8, G))]},
            "next_pass_us_by_lateness": follow,
            "seen_to_next_publish_min_us": round(float(np.median(gap)), 3)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--m", type=int, default=95)
    ap.add_argument("--steps", default="16,48,80")
    ap.add_argument("--tune", action="append", default=[], help="K=V: a GK_TUNE_* knob (e.g. 23=4, the blocked step)")
    a = ap.parse_args()
    import gmres_amd as ga

    with ga.Context(a.grid, a.m) as c:
        c.set_rhs_ones()
        for kv in a.tune:
            k, v = kv.split("=")
            c.tune(int(k), int(v))

        def run():
            return ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)

        run()  # warm
        for j in [int(s) for s in a.steps.split(",")]:
            c.zero_x()
            c.res_trace(1, j, 0)
            run()
            c.sync()
            pub, seen = c.res_trace(-1)
            c.res_trace(0)
            out = {"grid": a.grid, "m": a.m, "j": j}
            out.update(analyse(pub, seen))
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
