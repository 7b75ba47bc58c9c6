#!/bin/bash
# round 5: the LDS prefetch cap of the blocked step per workgroup (GK_BLK_PFX_KB: 128 main,
# 96 / 80 variants) at the small slabs (1024^2, 1448^2; S = 2 and 4), on the tree with the
# streamed tail on the last workgroup; bench lines alternating twice.
OUT=gpurun_out/r05ae
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
V=$PWD/gmres_amd/lib/variants
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
for k in 1 2; do
  for v in base kb96 kb80; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    for pt in "1448 4" "1448 2" "1024 4" "1024 2"; do
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
