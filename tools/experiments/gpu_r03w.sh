# Round 3: fewer workgroups for the resident step on small slabs?  GK_TUNE_RES_SHARE
# (10) = s makes the resident launches use CUs / s workgroups: 1024^2 and 2048^2
# (the per-rank slab of 4096^2 on 16 / 4 GPUs), s = 1, 2, 4.
OUT=gpurun_out/r03w
source tools/gpu_lib.sh
for g in 1024 2048; do
  for s in 1 2 4; do
    step g${g}_s${s} 200 python -u bench.py --no-cpu --no-configs --no-diag --steps 5 --warmup 2 --grid $g --tune 10=$s
  done
done
echo ALL_DONE
