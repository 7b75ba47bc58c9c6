#!/bin/bash
# round 5: the blocked step's ragged-tail element held in registers (w, the cached block, the
# next dot block loaded with the LDS prefetch during the all-gather) vs streamed in the pass
# (variant tail0): blocked tests first, then a trace and bench lines at 1448^2 (S = 2, 4) and
# 1024^2 (S = 4; no tail there: control), alternating twice.
OUT=gpurun_out/r05ah
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
V=$PWD/gmres_amd/lib/variants
step t_blk 600 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_blocked.py
tail -2 $OUT/t_blk.out
step tr_s4 200 python -u tools/res_trace.py --grid 1448 --tune 23=4
cut -c1-400 $OUT/tr_s4.out
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
for k in 1 2; do
  for v in base tail0; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    for pt in "1448 4" "1448 2" "1024 4"; do
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
