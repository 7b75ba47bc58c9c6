#!/bin/bash
# round 5: prefetch depth of the one-wave S = 4 blocked build at the 4096^2 / 8 load (1448^2):
# the first 8 (main) vs 9 / 6 of its 16 chunks of the next dot block into LDS during the
# all-gather; parity of the 9-chunk build first, then bench lines alternating twice.
OUT=gpurun_out/r05aa
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
V=$PWD/gmres_amd/lib/variants
GK_LIB_DIR=$V/s4pf9 step t_var 600 $T tests/test_gpu_blocked.py -k "4 and (instantiation or 1024_twelve or ragged or row_block)"
grep -E "passed|failed" $OUT/t_var.out | tail -3
for k in 1 2; do
  for v in base s4pf9 s4pf6; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    step b_${v}_$k 150 $B --grid 1448 --tune 23=4
    python - $OUT/b_${v}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 1), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"])
PY
  done
done
unset GK_LIB_DIR
echo ALL_DONE
