#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate passes,
MI355X_MICROARCH.md §HBM) into profiles/pmc_traffic.json, which bench.py
quotes as roofline.traffic for the matching workload.

gfx950 corrections applied (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half
the bytes of a wide coalesced streaming read -> x2; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Both derive from the L2's memory-side
requests, so Infinity-Cache hits are included: the figure is L2<->fabric
traffic (an upper bound on HBM traffic).

  python tools/pmc_summary.py --fetch F.csv --write W.csv --grid 4096 --m 95 \
      --prec identity --method mgsr --gpus 1 --kernel "gk::k_proj<2"
"""
import argparse
import csv
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    return statistics.median(vals) * 1024.0, len(vals)  # counters are in KB


def series(path, kernel):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [float(r["Counter_Value"]) * 1024.0 for r in rows]


def res_fit(a):
    """Per-launch bytes of the resident step kernel over ONE full cycle
    (bench.py --steps 1 --warmup 0: launches j = 1..m in dispatch order):
    recorded per step j (bench.py quotes the steps it samples, j % 16 == 0)
    plus a least-squares line fixed + per_projection * 2j with its residual."""
    import numpy as np

    f = np.array(series(a.fetch, a.kernel)) * 2.0  # gfx950 FETCH_SIZE correction
    w = np.array(series(a.write, a.kernel))
    k = min(len(f), len(w))
    if k < a.probe_m:
        raise SystemExit(f"only {k} launches of {a.kernel!r} (expected {a.probe_m})")
    y = f[: a.probe_m] + w[: a.probe_m]
    js = np.arange(1, a.probe_m + 1)
    b, c = np.polyfit(2 * js, y, 1)
    n = a.grid * a.grid // a.gpus
    # the byte model of the variant that ran (bench.res_launch_bytes, the roofline's)
    import sys

    sys.path.insert(0, ROOT)
    import bench
    import gmres_amd as ga

    nl = max(k for _, k in ga.slab_partition(a.grid, a.gpus))
    plan = ga.res_plan_query(a.grid * nl, 256, 1, a.method == "hh", -1, block=a.block)
    if a.variant and plan["variant"] != a.variant:
        raise SystemExit(f"the plan query selects {plan['variant']}, not {a.variant}")
    model = {int(j): bench.res_launch_bytes(plan, n, 2 * int(j), mgs=True) for j in js}
    entry = {"kernel": a.kernel, "variant": plan["variant"], "nloc": n, "G": int(plan["G"]),
             "launches_sampled": int(a.probe_m),
             "bytes_fixed": float(c),
             "bytes_per_projection": float(b), "bytes_per_unknown_per_projection": float(b) / n,
             "fit_residual_max_rel": float(np.max(np.abs(y - (b * 2 * js + c)) / y)),
             "per_step": {str(int(j)): float(v) for j, v in zip(js, y)},
             "per_step_model_ratio": {str(int(j)): float(v / model[int(j)]) for j, v in zip(js, y) if j % 16 == 0},
             "source": f"{os.path.relpath(a.fetch)} + {os.path.relpath(a.write)} (every launch j = 1..{a.probe_m} "
                       "of one full cycle, FETCH_SIZE x2 gfx950 correction; L2<->fabric bytes incl. "
                       "Infinity-Cache hits)"}
    db = json.load(open(a.out)) if os.path.exists(a.out) else {}
    pvar = f"blocked{a.block}" if plan["variant"] == "blocked" else plan["variant"]  # (bench.roofline_entry)
    entry["projection_block"] = a.block
    db[bench.pmc_key(pvar, n, a.m, a.prec, a.method)] = entry
    json.dump(db, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in entry.items() if k != "per_step"}, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--m", type=int, default=95)
    ap.add_argument("--prec", default="identity")
    ap.add_argument("--method", default="mgsr")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--kernel", default="gk::k_proj<2")
    ap.add_argument("--res", action="store_true",
                    help="resident-step kernel (one launch per Arnoldi step j = 1..probe-m in launch order): "
                         "fit bytes per launch = fixed + per_projection * 2j")
    ap.add_argument("--probe-m", type=int, default=95, help="resident launches of the traced cycle (= m)")
    ap.add_argument("--variant", default=None, help="the resident variant expected to have run (checked)")
    ap.add_argument("--block", type=int, default=1, help="GK_TUNE_RES_BLOCK of the traced run (blocked step: 2 / 4)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    if a.res:
        return res_fit(a)
    f, nf = per_launch(a.fetch, a.kernel)
    w, nw = per_launch(a.write, a.kernel)
    n = a.grid * a.grid // a.gpus
    entry = {"kernel": a.kernel, "launches_sampled": [nf, nw],
             "fetch_bytes_raw": f, "fetch_bytes_corrected": 2 * f, "write_bytes": w,
             "hbm_bytes_per_launch": 2 * f + w, "bytes_per_unknown": (2 * f + w) / n,
             "source": f"{os.path.relpath(a.fetch)} + {os.path.relpath(a.write)} (median per launch, "
                       "FETCH_SIZE x2 gfx950 correction; L2<->fabric bytes incl. Infinity-Cache hits)"}
    db = json.load(open(a.out)) if os.path.exists(a.out) else {}
    db[f"{a.grid}_{a.m}_{a.prec}_{a.method}_{a.gpus}"] = entry
    json.dump(db, open(a.out, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
