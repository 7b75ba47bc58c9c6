#!/bin/bash
# round 5: the strict MGS-R step on the blocked kernel with blocks of 1 and the LDS prefetch of the
# next dot column (GK_TUNE_RES_PF 1) against the strict kernels, at the per-GPU loads.
OUT=gpurun_out/r05w
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
step t_pf 600 $T tests/test_gpu_blocked.py -k "strict_prefetch"
grep -E "\[strict|passed|failed|Error" $OUT/t_pf.out | tail -10
grep -q " failed\|rror" $OUT/t_pf.out && { echo "pf tests failed"; exit 0; }
for k in 1 2; do
  for g in 1024 1448 2048 2896; do
    for v in strict pf; do
      if [ $v = pf ]; then a="--tune 27=1"; else a=""; fi
      step b_${g}_${v}_$k 150 $B --grid $g $a
      python - $OUT/b_${g}_${v}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"], d["roofline"]["variant"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
    done
  done
done
echo ALL_DONE
