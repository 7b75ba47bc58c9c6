# Round 3: fewer workgroups for the resident step on small slabs, resident
# launches forced on (GK_TUNE_RES 8 = 1: auto mode turns them off when
# RES_SHARE > 1) -- 1024^2 and 2048^2, s = 2, 4, 8, against the default plan.
# (Call w, the same without forcing the resident launches, did not get a box.)
OUT=gpurun_out/r03x
source tools/gpu_lib.sh
for g in 1024 2048; do
  step g${g}_base 200 python -u bench.py --no-cpu --no-configs --no-diag --steps 5 --warmup 2 --grid $g
  for s in 2 4 8; do
    step g${g}_s${s} 200 python -u bench.py --no-cpu --no-configs --no-diag --steps 5 --warmup 2 --grid $g --tune 8=1 --tune 10=$s
  done
done
echo ALL_DONE
