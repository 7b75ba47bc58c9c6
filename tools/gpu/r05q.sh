#!/bin/bash
# round 5: look-ahead blocked step, one wave per SIMD (256 threads, 8 / 16 register chunks,
# batch 8): tests, trace, then 1024^2 / 1448^2 against the plain blocked step S = 2 / 4.
OUT=gpurun_out/r05q
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
step t_la 600 $T tests/test_gpu_blocked.py -k "lookahead"
grep -E "look-ahead|passed|failed|Error" $OUT/t_la.out | tail -12
grep -q " failed\|error" $OUT/t_la.out && { echo "look-ahead tests failed"; exit 0; }
step trace 300 python -u tools/la_trace.py --grid 1448 --steps 32,80
cat $OUT/trace.out
for k in 1 2; do
  for g in 1024 1448; do
    for v in s2 s4 la; do
      case $v in
        s2) a="--tune 23=2";; s4) a="--tune 23=4";; la) a="--tune 23=2 --tune 26=1";;
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
echo ALL_DONE
