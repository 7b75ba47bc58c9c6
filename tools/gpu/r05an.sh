#!/bin/bash
# round 5: fewer producers for the all-gather-bound small slabs -- the resident launch on
# 256 / 128 / 64 workgroups (GK_TUNE_RES 1 + GK_TUNE_RES_SHARE 1 / 2 / 4) at 1024^2 (strict,
# blocked S = 4) and 1448^2 (blocked S = 4), alternating twice.
OUT=gpurun_out/r05an2
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
for k in 1 2; do
  for sh in 1 2 4; do
    for pt in "1024 1" "1024 4" "1448 4"; do
      set -- $pt
      step b_sh${sh}_$1_s$2_$k 150 $B --grid $1 --tune 23=$2 --tune 8=1 --tune 10=$sh
      python - $OUT/b_sh${sh}_$1_s$2_$k.out <<'PY' || true
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sp = (d["diagnostics"].get("resident_split_per_unit_us") or {}).get("mgs_step")
print(sys.argv[1].split('/')[-1], round(d["value"], 1), (d.get("roofline") or {}).get("per_projection_us"),
      d["config"]["resident_variant"], d["config"]["resident_workgroups"], sp)
PY
    done
  done
done
echo ALL_DONE
