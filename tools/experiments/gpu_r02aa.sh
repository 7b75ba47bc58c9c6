# Round 2, session E: replicated rank totals + per-kernel poll sleep: full GPU suite (incl.
# the device-exchange tests that run the resident step across contexts / processes), then
# A/B of the small-kernel poll sleep (s1 / s8 vs 4), 16 replicas, the flat sweep at 1024^2
# (hop1) and the big kernel's sleep (big8 vs 16).
OUT=gpurun_out/r02aa
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step ab1024 500 python -u tools/ab_lib.py --variants base s1 s8 rep16 hop1 --rounds 2 -- --steps 10 --warmup 2 --no-diag --grid 1024
step ab2048 500 python -u tools/ab_lib.py --variants base s1 s8 rep16 --rounds 2 -- --steps 5 --warmup 1 --no-diag --grid 2048
step ab4096 600 python -u tools/ab_lib.py --variants base rep16 big8 --rounds 2 -- --steps 3 --warmup 1 --no-diag
step trace4096 300 python -u tools/res_trace.py --grid 4096 --steps 48
echo ALL_DONE
