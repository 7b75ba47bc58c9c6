# Round 2, session E: paced, stoppable L2 touch-prefetch (GK_RES_TOUCH_PACE) A/B at 4096^2
# (MGS-R and Householder) against the all-at-once touch; interleaved chunk assignment (GK_RES_ILV);
# base2 = the current source rebuilt with default knobs.
OUT=gpurun_out/r02ac
source tools/gpu_lib.sh
step ab4096 600 python -u tools/ab_lib.py --variants base base2 pace8 pace24 touch48p ilv ilvpace8 --rounds 2 -- --steps 3 --warmup 1 --no-diag
step ab4096hh 600 python -u tools/ab_lib.py --variants base pace8 ilv --rounds 2 -- --steps 3 --warmup 1 --no-diag --method hh
echo ALL_DONE
