#!/bin/bash
# round 5: all-gather anatomy (tools/res_trace.py: arrival skew vs propagation) at the
# 4096^2 / 8 load (1448^2): strict, blocked S = 4 (main: 8 of 16 chunks prefetched) and
# blocked S = 4 without the prefetch (variant s4pf0), steps 16 / 48 / 80 of a warm cycle.
OUT=gpurun_out/r05ac
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
V=$PWD/gmres_amd/lib/variants
R="python -u tools/res_trace.py --grid 1448"
step tr_strict 200 $R
step tr_s4 200 $R --tune 23=4
GK_LIB_DIR=$V/s4pf0 step tr_s4pf0 200 $R --tune 23=4
GK_LIB_DIR=$V/s4pf6 step tr_s4pf6 200 $R --tune 23=4
for f in tr_strict tr_s4 tr_s4pf0 tr_s4pf6; do echo "== $f"; cat $OUT/$f.out; done
echo ALL_DONE
