# Round 2, session E: touch pacing re-tune after the depth / residency changes: Householder
# chains paced (8, 24) vs burst; MGS-R pace 16 / 32 vs 24.
OUT=gpurun_out/r02an
source tools/gpu_lib.sh
step ab4096hh 600 python -u tools/ab_lib.py --variants base hp8 hp24 --rounds 3 -- --steps 3 --warmup 1 --no-diag --method hh
step ab4096 600 python -u tools/ab_lib.py --variants base mp16 mp32 --rounds 3 -- --steps 3 --warmup 1 --no-diag
echo ALL_DONE
