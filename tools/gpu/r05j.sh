#!/bin/bash
# round 5, VERDICT r04 item 4: several rank-total pushers (GK_RES_PUSHERS 4 / 8,
# variant builds) against one (main build): the split tests on the variants, then
# same-device rehearsals -- 2 ranks at 1448^2, 4 ranks at 2048^2, 2 ranks at 2896^2 --
# alternating, three samples each.
OUT=gpurun_out/r05j
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
V=$PWD/gmres_amd/lib/variants
for v in p4 p8; do
  GK_LIB_DIR=$V/$v step splits_$v 600 $T tests/test_gpu_splits.py tests/test_gpu_blocked.py
  tail -2 $OUT/splits_$v.out
done
for k in 1 2 3; do
  for v in base p4 p8; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    step reh2_1448_${v}_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 1448
    step reh4_2048_${v}_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
    step reh2_2896_${v}_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
  done
done
unset GK_LIB_DIR
echo ALL_DONE
