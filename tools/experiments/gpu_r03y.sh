# Round 3: the Arnoldi step's stencil (w = A V(:,j) with the first dot's partials,
# 69.5 us = 5.8 TB/s at 4096^2): stencil workgroup target (GK_TUNE_STENCIL_BLOCKS 2)
# 2048 (default) vs 1024 / 4096 / 8192, kernel statistics of each.
OUT=gpurun_out/r03y
source tools/gpu_lib.sh
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for b in 2048 1024 4096 8192; do
  step st_$b 300 rocprofv3 --kernel-trace --stats -d $OUT/st_$b -o st --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag --tune 2=$b
done
echo ALL_DONE
