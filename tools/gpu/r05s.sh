#!/bin/bash
# round 5: the 4096^2 w-only step's touch extended into the Infinity Cache (device-scope
# loads past the 28 L2-touched chunks): 0 (main) / 32 / 60 chunks, alternating, three rounds.
OUT=gpurun_out/r05s
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
B="python -u bench.py --no-cpu --no-configs"
V=$PWD/gmres_amd/lib/variants
for k in 1 2 3; do
  for v in base tm32 tm60; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    step ab_${v}_$k 150 $B
    python - $OUT/ab_${v}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 2), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"], d["check"]["pass"])
PY
  done
done
echo ALL_DONE
