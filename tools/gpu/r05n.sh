#!/bin/bash
# round 5: look-ahead blocked step, 8-chunk build with slot set B in LDS (batch 4, main;
# batch 8, variant la8) -- tests, then 1448^2 / 1024^2 against the plain blocked step.
OUT=gpurun_out/r05n
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
V=$PWD/gmres_amd/lib/variants
step t_la 600 $T tests/test_gpu_blocked.py -k "lookahead"
grep -E "look-ahead|passed|failed|Error" $OUT/t_la.out | tail -12
grep -q " failed\|error" $OUT/t_la.out && { echo "look-ahead tests failed"; exit 0; }
GK_LIB_DIR=$V/la8 step t_la8 600 $T tests/test_gpu_blocked.py -k "lookahead"
tail -1 $OUT/t_la8.out
for k in 1 2; do
  for g in 1448 1024; do
    for v in s4 la la8; do
      case $v in
        s4) a="--tune 23=4"; unset GK_LIB_DIR;; la) a="--tune 23=2 --tune 26=1"; unset GK_LIB_DIR;;
        la8) a="--tune 23=2 --tune 26=1"; export GK_LIB_DIR=$V/la8;;
      esac
      step b_${g}_${v}_$k 150 $B --grid $g $a
      python - $OUT/b_${g}_${v}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
    done
  done
done
unset GK_LIB_DIR
echo ALL_DONE
