#!/bin/bash
# round 5: r05y's 8-rank leg again, now with one hardware queue per rank process
# (bench.py rank_env overrides the box's GPU_MAX_HW_QUEUES=4 in the same-device
# rehearsal; r05y's 8 x 4 queues time-sliced the warmup to 100 s and the silence
# guard ended it), then the 2- and 4-rank legs once more under the same queue count.
# Strict vs S = 2 / 4, alternating.
OUT=gpurun_out/r05y2
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
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["config"].get("resident_variant"),
      d["diagnostics"]["resident_split_per_unit_us"].get("mgs_step"), d.get("fallback"))
PY
}
for k in 1 2; do
  for s in 1 2 4; do
    step reh8_1448_s${s}_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 8 --grid 1448 --steps 2 --warmup 1 \
      --collective xgmi --tune 24=60000 --tune 23=$s
    show reh8_1448_s${s}_$k
  done
done
for cfg in "2 2896" "4 2048" "2 1448"; do
  set -- $cfg
  for s in 1 2 4; do
    step reh$1_$2_s${s}_q1 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus $1 --grid $2 --tune 23=$s
    show reh$1_$2_s${s}_q1
  done
done
echo ALL_DONE
