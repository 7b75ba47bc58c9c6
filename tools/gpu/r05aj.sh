#!/bin/bash
# round 5: the N-rank bench line's blocked leg (diagnostics.blocked_leg, after the timed region)
# in same-device rehearsals: 2 ranks at 1448^2 (S = 4), 4 ranks at 2048^2 (S = 2), 8 ranks at
# 1448^2 (S = 4; one queue per rank, 2 cycles).
OUT=gpurun_out/r05aj
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
( while sleep 45; do date +%T >> $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python -u bench.py --no-cpu --no-configs"
show() {
  python - $OUT/$1.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g = d["diagnostics"]
bl = g.get("blocked_leg") or {}
print(sys.argv[1].split('/')[-1], "strict", round(d["value"], 1), d["config"].get("resident_variant"),
      g["resident_split_per_unit_us"].get("mgs_step"), "| blocked S", bl.get("projection_block"), bl.get("it_s"),
      bl.get("resident_variant"), (bl.get("resident_split_per_unit_us") or {}).get("mgs_step"),
      (bl.get("check") or {}).get("rel_dev"), bl.get("error"))
PY
}
step reh2_1448 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 1448
show reh2_1448
step reh4_2048 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
show reh4_2048
step reh8_1448 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 8 --grid 1448 --steps 2 --warmup 1 --collective xgmi --tune 24=60000
show reh8_1448
echo ALL_DONE
