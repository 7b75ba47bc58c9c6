#!/bin/bash
# round 5: rocprofv3 kernel stats of the strict step at the 4- and 8-GPU loads (2048^2, 1448^2):
# the default kernels vs the prefetching blocked kernel with blocks of 1 (GK_TUNE_RES_PF 1).
OUT=gpurun_out/r05as
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
for g in 2048 1448; do
  for pf in 0 1; do
    step tr_${g}_pf$pf 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_${g}_pf$pf" -o k --output-format csv -- python3 bench.py --grid $g --tune 27=$pf --steps 3 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
    head -3 $OUT/tr_${g}_pf$pf/k_kernel_stats.csv | cut -c1-160
  done
done
echo ALL_DONE
