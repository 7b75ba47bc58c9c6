#!/usr/bin/env python3
"""Read a driver scaling file (SCALE_rNN.json) against the committed prediction
(profiles/r04/scaling_prediction_r04.json, tools/predict_scaling.py).

The driver's file format is not fixed here: every bench line found anywhere in
it (a JSON object with "metric" and "n_gpus", possibly inside a stdout tail
string) is taken, and for each world size the measured it/s, the per-projection
wait of the resident step and the collective per-call latency are set beside
the predicted band.

  python tools/read_scale.py SCALE_r05.json [--pred profiles/r04/scaling_prediction_r04.json]
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


def compare(lines: list[dict], pred: dict) -> list[dict]:
    rows = []
    by_world = {p["world"]: p for p in pred["points"] if p.get("grid") == 4096 and "world" in p}
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
        rows.append({"n_gpus": n, "it_s": b["value"], "predicted_it_s": [lo, hi], "verdict": verdict,
                     "variant": (b.get("config") or {}).get("resident_variant"),
                     "collective": (b.get("config") or {}).get("collective"),
                     "wait_us": wait, "predicted_wait_us": wlo,
                     "collective_latency_us": d.get("collective_latency_us")})
    return rows


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("scale")
    ap.add_argument("--pred", default=os.path.join(ROOT, "profiles", "r04", "scaling_prediction_r04.json"))
    a = ap.parse_args()
    rows = compare(bench_lines(json.load(open(a.scale))), json.load(open(a.pred)))
    print("| N | it/s | predicted | verdict | variant | collective | wait us (pred) | collective us |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['n_gpus']} | {r['it_s']} | {r['predicted_it_s']} | {r['verdict']} | {r['variant']} | "
              f"{r['collective']} | {r['wait_us']} ({r['predicted_wait_us']}) | {r['collective_latency_us']} |")


if __name__ == "__main__":
    main()
