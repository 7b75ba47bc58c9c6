#!/bin/bash
# round 5: blocks of 8 on the smallest slabs (1024^2: one wave per SIMD, 8 cached columns).
# Blocked tests first; then 1024^2 lines S = 4 vs 8 alternating twice, a 2-rank 1024^2
# rehearsal with S = 8, and the default bench line.
OUT=gpurun_out/r05ao
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
step t_blk 600 python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_blocked.py
grep -E "blocked S=8|PASS|FAIL" $OUT/t_blk.out | grep -E "S=8|FAIL" | head -20; tail -1 $OUT/t_blk.out
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
for k in 1 2; do
  for s in 4 8; do
    step b_1024_s${s}_$k 150 $B --grid 1024 --tune 23=$s
    python - $OUT/b_1024_s${s}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"], d["roofline"]["frac"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"], d["check"].get("rel_dev"))
PY
  done
done
step reh2_1024_s8 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 1024 --tune 23=8
tail -c 400 $OUT/reh2_1024_s8.out
echo ALL_DONE
