# Round 2, session D: all-gather polling A/B -- serialized polls (HEAD), parallel polls
# with s_sleep 1 (base) / 4 / 16 / 48 between unanswered polls; 4096^2 and 1024^2.
OUT=gpurun_out/r02m
source tools/gpu_lib.sh
step ab4096 900 python -u tools/ab_lib.py --variants base serial sl4 sl16 sl48 --rounds 2 -- --steps 3 --warmup 1 --no-diag
step ab1024 900 python -u tools/ab_lib.py --variants base serial sl4 sl16 sl48 --rounds 2 -- --steps 10 --warmup 2 --grid 1024 --no-diag
echo ALL_DONE
