#!/bin/bash
# round 5: the default 4096^2 line with the streamed tail on the last workgroup (main) vs
# the round-4 assignment (variant swg0): r05af's default line came in at 246.6 it/s against
# 252.6 in r05x -- a box, or the change?  Alternating three times on one box.
OUT=gpurun_out/r05ag
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
V=$PWD/gmres_amd/lib/variants
B="python -u bench.py --no-cpu --no-configs --steps 3 --warmup 1"
for k in 1 2 3; do
  for v in base swg0; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    step b_${v}_$k 200 $B
    python - $OUT/b_${v}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
  done
done
echo ALL_DONE
