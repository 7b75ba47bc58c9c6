#!/bin/bash
# round 5: the blocked step's poll interval (GK_BLK_POLL_SLEEP: s_sleep 16 main vs 4 / 8 / 32
# variants) at 1024^2 S = 4 and 1448^2 S = 4 / 2, alternating twice.
OUT=gpurun_out/r05al
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
V=$PWD/gmres_amd/lib/variants
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
for k in 1 2; do
  for v in base sl4 sl8 sl32; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    for pt in "1024 4" "1448 4" "1448 2"; do
      set -- $pt
      step b_${v}_$1_s$2_$k 150 $B --grid $1 --tune 23=$2
      python - $OUT/b_${v}_$1_s$2_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
    done
  done
done
echo ALL_DONE
