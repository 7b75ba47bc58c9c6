#!/bin/bash
# round 5: the LDS ring of the one-wave S = 4 blocked build (the 4096^2 / 8 load): the dot
# block streams through 9 LDS slots by LDS-DMA, 6 prefetched during the all-gather, chunk
# k + 9 issued as chunk k is read.  Blocked tests first; then 1448^2 S = 4 lines against the
# register-batch build (variant ring0), alternating twice, and a trace.
OUT=gpurun_out/r05ai
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
V=$PWD/gmres_amd/lib/variants
step t_blk 600 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_blocked.py
grep -E "PASS|FAIL" $OUT/t_blk.out | grep -c PASS; grep -E "FAILED" $OUT/t_blk.out | head; tail -2 $OUT/t_blk.out
B="python -u bench.py --no-cpu --no-configs --steps 4 --warmup 1"
for k in 1 2; do
  for v in base ring0; do
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
step tr_s4 200 python -u tools/res_trace.py --grid 1448 --tune 23=4
cut -c1-300 $OUT/tr_s4.out
echo ALL_DONE
