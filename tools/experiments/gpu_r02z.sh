# Round 2, session E: replicated granule arrays for the in-launch all-gather (GK_RES_NREP):
# full GPU suite on the new default (8 replicas), all-gather anatomy, and an interleaved
# A/B against one array (rep1), a shorter poll sleep (rep8s4) and the session's starting
# library (head) at 4096^2, 2048^2, 1024^2.
OUT=gpurun_out/r02z
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step trace4096 300 python -u tools/res_trace.py --grid 4096 --steps 16,48,80
step trace1024 300 python -u tools/res_trace.py --grid 1024 --steps 16,48,80
step ab4096 600 python -u tools/ab_lib.py --variants base rep1 rep8s4 head --rounds 2 -- --steps 3 --warmup 1 --no-diag
step ab2048 400 python -u tools/ab_lib.py --variants base rep1 rep8s4 head --rounds 2 -- --steps 5 --warmup 1 --no-diag --grid 2048
step ab1024 400 python -u tools/ab_lib.py --variants base rep1 rep8s4 head --rounds 2 -- --steps 10 --warmup 2 --no-diag --grid 1024
echo ALL_DONE
