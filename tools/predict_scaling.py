#!/usr/bin/env python3
"""A falsifiable prediction of the strong-scaling curve (4096^2 on 1/2/4/8 GPUs)
and of config 4 (8192^2 on 8 GPUs), regenerated from committed single-GPU
measurements.

Model.  An N-rank run gives every GPU a slab of n/N unknowns; its Arnoldi steps
run the resident kernel that slab selects (tests/test_res_plan.py), on all 256
CUs, exactly as a single-GPU run of a grid with the same unknown count does
(1448^2 ~ 4096^2/8, 2048^2 ~ 4096^2/4, 2896^2 ~ 4096^2/2 and 8192^2/8).  So the
per-GPU cycle time is that single-GPU cycle (bench.py --grid G, ms_per_step)
plus what only N ranks pay:
  * per Arnoldi step, one collective launch on the step's critical path: the
    halo lines before the stencil (k_xhalo), priced at gk_comm_latency's
    per-call time (the stencil's first dot is summed across ranks inside the
    resident launch, GK_TUNE_RES_FOLD: one more in-launch hop per step);
  * per projection (and per step for the first dot), the hop of the rank totals
    inside the resident launch (workgroup 0 of every rank stores its total into
    every peer's region over xGMI, every workgroup polls its own region): delta_hop.
  t_cycle(N) = t_cycle_1GPU(n/N) + m t_halo + m (m + 2) delta_hop
  it/s(N)    = m / t_cycle(N),  value of the N-GPU bench line (max over ranks).
Bands.  The collective per-call time at the high end is gk_comm_latency of the
same-device rehearsal (N processes on ONE GPU through IPC, back-to-back calls:
launch gaps and N-process contention included, no xGMI crossing); at the low
end --coll-lo (default 5 us: the exchange's round trip with the launch hidden
behind the queued step, as in the solve).  delta_hop is bracketed by
[--hop-lo, --hop-hi] (default 1..4 us: one uncached store crossing xGMI and a
poll).
Each SCALE line carries diagnostics.resident_split_per_unit_us (the measured
wait per projection) and collective_latency_us, against which the predicted
terms can be read directly.

  python tools/predict_scaling.py [--hop-lo 1.0] [--hop-hi 4.0] [--out profiles/r04/scaling_prediction_r04.json]
"""
from __future__ import annotations

import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M = 95

# per-GPU load of each point -> the single-GPU bench line measured at that load
POINTS = [
    # (label, world, global grid, equal-load single-GPU grid, bench JSON under profiles/)
    ("4096^2 on 1 GPU", 1, 4096, 4096, "r05/bench_point_4096_strict_r05z2.json"),
    ("4096^2 on 2 GPUs", 2, 4096, 2896, "r05/bench_point_2896_strict_r05z2.json"),
    ("4096^2 on 4 GPUs", 4, 4096, 2048, "r05/bench_point_2048_strict_r05z2.json"),
    ("4096^2 on 8 GPUs", 8, 4096, 1448, "r05/bench_point_1448_strict_r05z2.json"),
    ("8192^2 on 8 GPUs (config 4)", 8, 8192, 2896, "r05/bench_point_2896_strict_r05z2.json"),
]
# the same points with the opt-in blocked-projection step (GK_TUNE_RES_BLOCK S, round 5):
# per point the block size that measured fastest at that load, one in-launch all-gather
# (and so one cross-rank hop) per block of S projections
POINTS_BLOCKED = [
    ("4096^2 on 1 GPU", 1, 4096, 4096, "r05/bench_point_4096_blk4_r05l.json", 4),
    ("4096^2 on 2 GPUs", 2, 4096, 2896, "r05/bench_point_2896_blk2_r05h.json", 2),
    ("4096^2 on 4 GPUs", 4, 4096, 2048, "r05/bench_point_2048_blk2_r05h.json", 2),
    ("4096^2 on 8 GPUs", 8, 4096, 1448, "r06/bench_point_1448_blk4_r06n.json", 4),
    ("8192^2 on 8 GPUs (config 4)", 8, 8192, 2896, "r05/bench_point_2896_blk2_r05h.json", 2),
]


def hops_per_cycle(S: int) -> int:
    """In-launch cross-rank hops of one cycle: per step the first dot's plus one per
    all-gather -- 2j (strict) or 2 (1 + ceil((j-1)/S)) (blocked, gk_blk.hpp)."""
    if S <= 1:
        return M * (M + 2)
    return sum(1 + 2 * (1 + (j - 1 + S - 1) // S) for j in range(1, M + 1))


# {"2": {"allreduce": us, "halo": us}, "4": {...}}: gk_comm_latency of same-device rehearsals
COMM = "r04/rehearsal_comm_latency_r04d.json"


def load(rel: str) -> dict | None:
    p = os.path.join(ROOT, "profiles", rel)
    if not os.path.exists(p):
        return None
    txt = open(p).read().strip()
    try:
        return json.loads(txt)
    except json.JSONDecodeError:
        return json.loads([x for x in txt.splitlines() if x.startswith("{")][-1])


def predict(hop_lo: float, hop_hi: float, coll_lo: float = 5.0, blocked: bool = False) -> dict:
    comm = load(COMM) or {}
    rows = []
    for pt in (POINTS_BLOCKED if blocked else POINTS):
        label, world, grid, g1, rel = pt[:5]
        S = pt[5] if blocked else 1
        cw = comm.get(str(world)) or comm.get(str(max([int(k) for k in comm if k.isdigit()] or [0]))) or {}
        t_ar, t_halo = float(cw.get("allreduce", 10.0)), float(cw.get("halo", 10.0))
        fixed_lo = 0.0 if world == 1 else M * coll_lo * 1e-6
        b = load(rel)
        if b is None:
            rows.append({"point": label, "missing": rel})
            continue
        t1 = float(b["ms_per_step"]) * 1e-3  # one cycle of the equal-load single-GPU run
        split = ((b.get("diagnostics") or {}).get("resident_split_per_unit_us") or {}).get("mgs_step") or {}
        extra_fixed = 0.0 if world == 1 else M * t_halo * 1e-6
        nproj = hops_per_cycle(S)  # strict: the 2j projections of every step plus its first dot
        lo = t1 + fixed_lo + (0.0 if world == 1 else nproj * hop_lo * 1e-6)
        hi = t1 + extra_fixed + (0.0 if world == 1 else nproj * hop_hi * 1e-6)
        rows.append({
            "point": label, "world": world, "grid": grid, "per_gpu_unknowns": grid * grid // world,
            "projection_block": S, "hops_per_cycle": nproj if world > 1 else 0,
            "equal_load_grid": g1, "variant": (b.get("config") or {}).get("resident_variant"),
            "t_cycle_1gpu_ms": round(t1 * 1e3, 2),
            "per_projection_1gpu_us": (b.get("roofline") or {}).get("per_projection_us"),
            "pass_us": split.get("pass_us"), "wait_us": split.get("wait_us"),
            "collective_per_call_us": {"allreduce": t_ar, "halo": t_halo} if world > 1 else None,
            "collective_ms_per_cycle": [round(fixed_lo * 1e3, 2), round(extra_fixed * 1e3, 2)],
            "hop_ms_per_cycle": [round(nproj * hop_lo * 1e-3, 2), round(nproj * hop_hi * 1e-3, 2)] if world > 1 else 0,
            "predicted_ms_per_cycle": [round(lo * 1e3, 1), round(hi * 1e3, 1)],
            "predicted_it_s": [round(M / hi, 1), round(M / lo, 1)],
            "predicted_wait_per_projection_us": ([round((split.get("wait_us") or 0) + hop_lo, 2),
                                                  round((split.get("wait_us") or 0) + hop_hi, 2)] if world > 1 else
                                                 split.get("wait_us")),
            "source": f"profiles/{rel}",
        })
    base = next((r for r in rows if r.get("world") == 1), None)
    for r in rows:
        if base and "predicted_it_s" in r and r["grid"] == 4096:
            r["predicted_speedup"] = [round(v / base["predicted_it_s"][1], 2) for v in r["predicted_it_s"]]
    return {"model": ("t_cycle(N) = t_cycle_1GPU(n/N) + m t_halo + hops delta_hop (first dot folded into the launch; "
                      "hops = m (m+2) strict, sum_j 1 + 2 (1 + ceil((j-1)/S)) blocked)"),
            "m": M, "collective_per_call_low_us": coll_lo, "collective_source": f"profiles/{COMM}" if comm else "default 10 us (no rehearsal file)",
            "delta_hop_us": [hop_lo, hop_hi], "points": rows}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hop-lo", type=float, default=1.0)
    ap.add_argument("--hop-hi", type=float, default=4.0)
    ap.add_argument("--coll-lo", type=float, default=5.0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06", "scaling_prediction_r06.json"))
    a = ap.parse_args()
    out = {"strict": predict(a.hop_lo, a.hop_hi, a.coll_lo),
           "blocked": predict(a.hop_lo, a.hop_hi, a.coll_lo, blocked=True)}
    json.dump(out, open(a.out, "w"), indent=1)
    for name, tab in out.items():
        print(f"\n{name}:")
        table(tab)


def table(out: dict) -> None:
    print("| point | variant (S) | 1-GPU cycle at the per-GPU load (ms) | predicted ms / cycle | predicted it/s |"
          " predicted wait / projection (us) |")
    print("|---|---|---|---|---|---|")
    for r in out["points"]:
        if "missing" in r:
            print(f"| {r['point']} | missing {r['missing']} | | | | |")
            continue
        print(f"| {r['point']} | {r['variant']} ({r['projection_block']}) | {r['t_cycle_1gpu_ms']} | "
              f"{r['predicted_ms_per_cycle'][0]}-"
              f"{r['predicted_ms_per_cycle'][1]} | {r['predicted_it_s'][0]}-{r['predicted_it_s'][1]} | "
              f"{r['predicted_wait_per_projection_us']} |")


if __name__ == "__main__":
    main()
