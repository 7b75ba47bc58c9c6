#!/usr/bin/env python3
"""All-gather anatomy of the look-ahead blocked step (k_mgs_bla) against the plain
blocked step: gk_profile_res_trace stamps, per workgroup and all-gather x, the
publish time and the moment the total was in hand.  In the look-ahead step x is
collected right after the workgroup published x + 1, so

  collect wait_g(x) = have_g(x) - pub_g(x + 1)    (the part not hidden by the pass)
  skew_g(x)         = max_g' pub_g'(x) - pub_g(x)
  prop(x)           = have_g(x) - max_g' pub_g'(x)

  python tools/la_trace.py --grid 1448 --steps 48
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1448)
    ap.add_argument("--steps", default="48")
    a = ap.parse_args()
    import gmres_amd as ga
    from gmres_amd import _native as nat

    for la in (0, 1):
        with ga.Context(a.grid, 95) as c:
            c.set_rhs_ones()
            c.tune(nat.GK_TUNE_RES_BLOCK, 2)
            c.tune(nat.GK_TUNE_RES_LOOKAHEAD, la)
            run = lambda: ga.gmres_mgsr(c, 1e-15, max_cycles=1, want_verr=False)  # noqa: E731
            run()
            for j in [int(s) for s in a.steps.split(",")]:
                c.zero_x()
                c.res_trace(1, j, 0)
                run()
                c.sync()
                pub, seen = c.res_trace(-1)
                c.res_trace(0)
                X = pub.shape[1]
                ok = [x for x in range(X) if (pub[:, x] > 0).all() and (seen[:, x] > 0).all()]
                pub, seen = pub[:, ok] * 1e3, seen[:, ok] * 1e3  # us
                last = pub.max(axis=0)
                out = {"grid": a.grid, "j": j, "lookahead": la, "exchanges": len(ok),
                       "skew_us": round(float((last[None, :] - pub).mean()), 3),
                       "spread_us": round(float((last - pub.min(axis=0)).mean()), 3),
                       "prop_us": round(float((seen - last[None, :]).mean()), 3),
                       "prop_min_us": round(float((seen - last[None, :]).min()), 3)}
                if la and pub.shape[1] > 1:
                    cw = seen[:, :-1] - pub[:, 1:]  # collect of x starts right after publishing x + 1
                    out["collect_wait_us"] = round(float(cw.mean()), 3)
                    out["pass_between_us"] = round(float((pub[:, 1:] - pub[:, :-1]).mean()), 3)
                else:
                    out["pass_between_us"] = round(float((pub[:, 1:] - seen[:, :-1]).mean()), 3)
                print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
