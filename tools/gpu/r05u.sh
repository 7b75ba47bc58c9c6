#!/bin/bash
# round 5: the one-wave S = 4 small-slab build as the default -- blocked tests, the split
# tests, and the 1448^2 / 1024^2 points.
OUT=gpurun_out/r05u
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
step t_blk 600 $T tests/test_gpu_blocked.py tests/test_gpu_configs.py -k "blocked or blk2"
grep -E "\[blocked|passed|failed" $OUT/t_blk.out | tail -30
for g in 1448 1024; do for s in 2 4; do
  step b_${g}_s$s 150 $B --grid $g --tune 23=$s
  tail -1 $OUT/b_${g}_s$s.out > $OUT/b_${g}_s$s.json
done; done
echo ALL_DONE
