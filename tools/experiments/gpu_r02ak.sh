# Round 2, session E: w residency / batch depth of the w-only step after the all-gather
# changes: RW 88 / WB 8 (base) vs WB 6, RW 89 and RW 90 with WB 6 (RW 90 + LW 38 = the
# whole 4096^2 slab on chip, nothing streamed), MGS-R and Householder.
OUT=gpurun_out/r02ak
source tools/gpu_lib.sh
step ab4096 600 python -u tools/ab_lib.py --variants base wb6 rw89wb6 rw90wb6 --rounds 3 -- --steps 3 --warmup 1 --no-diag
step ab4096hh 600 python -u tools/ab_lib.py --variants base rw90wb6 --rounds 2 -- --steps 3 --warmup 1 --no-diag --method hh
echo ALL_DONE
