#!/bin/bash
# round 5: blocked step S = 2 at the 4096^2 / 4 load (2048^2): one-wave build (256 threads, 32
# chunks of w and both cached columns in registers, 16 chunks of the next dot block prefetched
# into LDS; variant s2r16w1) vs the two-wave build (7 + 9 of 16 chunks cached, main), strict beside.
OUT=gpurun_out/r05v
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
V=$PWD/gmres_amd/lib/variants
GK_LIB_DIR=$V/s2r16w1 step t_var 600 $T tests/test_gpu_blocked.py -k "2 and (1024_twelve or ragged or row_block or 4096)"
grep -E "\[blocked S=2|passed|failed" $OUT/t_var.out | tail -12
for k in 1 2; do
  for v in base s2r16w1; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    for s in 2 1; do
      step b_${v}_s${s}_$k 150 $B --grid 2048 --tune 23=$s
      python - $OUT/b_${v}_s${s}_$k.out <<'PY'
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
