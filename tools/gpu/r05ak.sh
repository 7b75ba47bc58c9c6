#!/bin/bash
# round 5: the blocked step's prefetch during an all-gather issued by the waves that do not poll
# it (GK_BLK_PF_SPLIT, the 512-thread builds) vs every wave its own elements (variant split0);
# and with the 128 KiB cap (variant split_kb128).  Blocked tests first, then 1024^2 S = 4 / 2
# and 1448^2 S = 2 / 4 lines alternating twice.
OUT=gpurun_out/r05ak
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
V=$PWD/gmres_amd/lib/variants
step t_blk 600 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_blocked.py
tail -1 $OUT/t_blk.out
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
for k in 1 2; do
  for v in base split0 split_kb128; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    for pt in "1024 4" "1024 2" "1448 2" "1448 4"; do
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
