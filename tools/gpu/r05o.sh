#!/bin/bash
# round 5: look-ahead blocked step -- the all-gather poll interval (s_sleep 16 main, 4 / 48
# variants) at 1024^2 and 1448^2, plain blocked S = 4 beside it.
OUT=gpurun_out/r05o
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
V=$PWD/gmres_amd/lib/variants
for k in 1 2; do
  for g in 1024 1448; do
    for v in base lap4 lap48; do
      if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
      for m in la s4; do
        if [ $m = la ]; then a="--tune 23=2 --tune 26=1"; else a="--tune 23=4"; fi
        step b_${g}_${v}_${m}_$k 150 $B --grid $g $a
        python - $OUT/b_${g}_${v}_${m}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
      done
    done
  done
done
unset GK_LIB_DIR
echo ALL_DONE
