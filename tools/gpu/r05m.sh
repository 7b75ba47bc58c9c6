#!/bin/bash
# round 5: the look-ahead blocked step (k_mgs_bla, GK_TUNE_RES_LOOKAHEAD 1 with S = 2):
# its GPU tests, then bench points at 1024^2 and 1448^2 against the plain blocked
# step (S = 2, 4) and strict MGS-R, alternating twice.
OUT=gpurun_out/r05m
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
step t_la 600 $T tests/test_gpu_blocked.py -k "lookahead"
grep -E "look-ahead|passed|failed|Error" $OUT/t_la.out | tail -12
grep -q " failed\|error" $OUT/t_la.out && { echo "look-ahead tests failed"; exit 0; }
for k in 1 2; do
  for g in 1024 1448; do
    for v in strict s2 s4 la; do
      case $v in
        strict) a="";; s2) a="--tune 23=2";; s4) a="--tune 23=4";; la) a="--tune 23=2 --tune 26=1";;
      esac
      step b_${g}_${v}_$k 150 $B --grid $g $a
      python - $OUT/b_${g}_${v}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"], d["check"]["pass"])
PY
    done
  done
done
echo ALL_DONE
