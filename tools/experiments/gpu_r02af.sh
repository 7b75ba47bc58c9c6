# Round 2, session E: L2 touch depth with paced touches (GK_RES_TOUCH 24 / 32 / 40 / 48 chunks).
OUT=gpurun_out/r02af
source tools/gpu_lib.sh
step ab4096 600 python -u tools/ab_lib.py --variants base t24 t40 t48 --rounds 3 -- --steps 3 --warmup 1 --no-diag
echo ALL_DONE
