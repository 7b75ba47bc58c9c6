# Round 2, session E: touch depth per launch kind -- MGS-R (paced) 16 / 20 / 24 / 28 chunks,
# Householder chains (burst) 24 vs 32.
OUT=gpurun_out/r02ag
source tools/gpu_lib.sh
step ab4096 600 python -u tools/ab_lib.py --variants base m16 m20 m28 --rounds 3 -- --steps 3 --warmup 1 --no-diag
step ab4096hh 400 python -u tools/ab_lib.py --variants base hh24 --rounds 3 -- --steps 3 --warmup 1 --no-diag --method hh
echo ALL_DONE
