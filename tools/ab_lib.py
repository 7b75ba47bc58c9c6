#!/usr/bin/env python3
"""A/B of library builds (gmres_amd/build.py build_variant) on one GPU box:
each variant's bench line is taken in its own process (GK_LIB_DIR selects the
build), variants interleaved over several rounds so box drift hits all alike.

  python tools/ab_lib.py --variants base xpf88 xpf80 --rounds 2 -- --steps 3 --warmup 1
  python tools/ab_lib.py --variants base tune:17=0 -- --steps 3    (a GK_TUNE_* knob of the base build)
Prints one JSON object per run and a summary (median it/s, per-projection us).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=240)
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    extra = [x for x in a.bench_args if x != "--"]
    res = {v: [] for v in a.variants}
    for r in range(a.rounds):
        for v in a.variants:
            env = dict(os.environ)
            tune = []
            if v.startswith("tune:"):  # a runtime knob of the base build: tune:KEY=VALUE[,KEY=VALUE]
                for kv in v[5:].split(","):
                    tune += ["--tune", kv]
            elif v != "base":
                env["GK_LIB_DIR"] = os.path.join(ROOT, "gmres_amd", "lib", "variants", v)
            p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", *tune, *extra],
                               capture_output=True, text=True, env=env, timeout=a.timeout)
            if p.returncode != 0:
                print(json.dumps({"variant": v, "round": r, "rc": p.returncode, "err": p.stderr[-800:]}), flush=True)
                if p.returncode not in (0, 1):
                    sys.exit(p.returncode)
                continue
            d = json.loads(p.stdout.strip().splitlines()[-1])
            roof = d.get("roofline") or {}
            row = {"variant": v, "round": r, "value": d["value"], "ms_per_step": d["ms_per_step"],
                   "per_projection_us": roof.get("per_projection_us"), "frac": roof.get("frac"),
                   "resid": d["check"]["true_rel_residual_after_timed_cycles"], "fallback": d.get("fallback"),
                   "split": ((d.get("diagnostics") or {}).get("resident_split_per_unit_us"))}
            res[v].append(row)
            print(json.dumps(row), flush=True)
    summ = {v: {"median_it_s": statistics.median([x["value"] for x in rows]),
                "median_proj_us": statistics.median([x["per_projection_us"] or 0 for x in rows])}
            for v, rows in res.items() if rows}
    print(json.dumps({"summary": summ, "bench_args": extra}), flush=True)


if __name__ == "__main__":
    main()
