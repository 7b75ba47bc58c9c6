#!/bin/bash
# round 5: the blocked step in same-device rehearsals (the in-launch rank hop per block of S):
# 2 ranks at 2896^2, 4 at 2048^2, 2 and 8 at 1448^2 -- strict vs S = 2 / 4, alternating twice.
OUT=gpurun_out/r05y
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
B="python -u bench.py --no-cpu --no-configs"
for k in 1 2; do
  for cfg in "2 2896" "4 2048" "2 1448" "8 1448"; do
    set -- $cfg
    for s in 1 2 4; do
      step reh$1_$2_s${s}_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus $1 --grid $2 --tune 23=$s
      python - $OUT/reh$1_$2_s${s}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["config"].get("resident_variant"),
      d["diagnostics"]["resident_split_per_unit_us"].get("mgs_step"), d.get("fallback"))
PY
    done
  done
done
echo ALL_DONE
