#!/usr/bin/env python3
"""Read a driver scaling file (SCALE_rNN.json) against the committed prediction
(profiles/r05/scaling_prediction_r05.json, tools/predict_scaling.py: a strict and a
blocked table; round 4's single table is read too).

The driver's file format is not fixed here: every bench line found anywhere in
it (a JSON object with "metric" and "n_gpus", possibly inside a stdout tail
string) is taken, and for each world size the measured it/s, the per-projection
wait of the resident step and the collective per-call latency are set beside
the predicted band -- and, where the line carries diagnostics.blocked_leg (N > 1,
round 5 on), the blocked step's it/s beside the blocked table.

  python tools/read_scale.py SCALE_r05.json [--pred profiles/r05/scaling_prediction_r05.json]
"""
from __future__ import annotations

import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_lines(obj) -> list[dict]:
    """Every bench line inside obj (dicts, lists, and JSON lines inside strings)."""
    out = []
    if isinstance(obj, dict):
        if "metric" in obj and "n_gpus" in obj and "value" in obj:
            out.append(obj)
        for v in obj.values():
            out += bench_lines(v)
    elif isinstance(obj, list):
        for v in obj:
            out += bench_lines(v)
    elif isinstance(obj, str) and '"metric"' in obj:
        for line in obj.splitlines():
            line = line.strip()
            if line.startswith("{"):
                try:
                    out += bench_lines(json.loads(line))
                except json.JSONDecodeError:
                    pass
    return out


def _band(v, band):
    lo, hi = band or (None, None)
    if v is None or lo is None:
        return None
    return "below band" if v < lo else ("above band" if v > hi else "inside band")


def compare(lines: list[dict], pred: dict) -> list[dict]:
    rows = []
    blocked = pred.get("blocked") or {}
    pred = pred.get("strict", pred)
    by_world = {p["world"]: p for p in pred["points"] if p.get("grid") == 4096 and "world" in p}
    blk_world = {p["world"]: p for p in blocked.get("points", []) if p.get("grid") == 4096 and "world" in p}
    for b in sorted(lines, key=lambda x: x["n_gpus"]):
        n = int(b["n_gpus"])
        p = by_world.get(n, {})
        d = b.get("diagnostics") or {}
        wait = ((d.get("resident_split_per_unit_us") or {}).get("mgs_step") or {}).get("wait_us")
        lo, hi = (p.get("predicted_it_s") or [None, None])
        wlo = p.get("predicted_wait_per_projection_us")
        verdict = None
        if lo is not None:
            verdict = "below band" if b["value"] < lo else ("above band" if b["value"] > hi else "inside band")
        bl = d.get("blocked_leg") or {}
        bp = blk_world.get(n, {})
        rows.append({"n_gpus": n, "it_s": b["value"], "predicted_it_s": [lo, hi], "verdict": verdict,
                     "variant": (b.get("config") or {}).get("resident_variant"),
                     "collective": (b.get("config") or {}).get("collective"),
                     "wait_us": wait, "predicted_wait_us": wlo,
                     "collective_latency_us": d.get("collective_latency_us"),
                     "blocked_it_s": bl.get("it_s"), "blocked_S": bl.get("projection_block"),
                     "blocked_predicted_it_s": bp.get("predicted_it_s"),
                     "blocked_verdict": _band(bl.get("it_s"), bp.get("predicted_it_s")),
                     "strict_prefetch_it_s": (d.get("strict_prefetch_leg") or {}).get("it_s")})
    return rows


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("scale")
    ap.add_argument("--pred", default=os.path.join(ROOT, "profiles", "r05", "scaling_prediction_r05.json"))
    a = ap.parse_args()
    rows = compare(bench_lines(json.load(open(a.scale))), json.load(open(a.pred)))
    print("| N | it/s | predicted | verdict | variant | collective | wait us (pred) | collective us |"
          " blocked leg it/s (S) | predicted | verdict | strict-prefetch leg it/s |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['n_gpus']} | {r['it_s']} | {r['predicted_it_s']} | {r['verdict']} | {r['variant']} | "
              f"{r['collective']} | {r['wait_us']} ({r['predicted_wait_us']}) | {r['collective_latency_us']} | "
              f"{r['blocked_it_s']} ({r['blocked_S']}) | {r['blocked_predicted_it_s']} | {r['blocked_verdict']} | "
              f"{r['strict_prefetch_it_s']} |")


if __name__ == "__main__":
    main()
