# Round 2, session D: touch-prefetch depth A/B (MGS-R and Householder), v_err reference-run band.
OUT=gpurun_out/r02f
source tools/gpu_lib.sh
step verr 300 python -u -m pytest tests/test_gpu_solver.py -v --timeout 200 --timeout-method thread -k verr
step ab_mgs 900 python -u tools/ab_lib.py --variants base touch32 touch48 touch64 --rounds 2 -- --steps 3 --warmup 1
step ab_hh 900 python -u tools/ab_lib.py --variants base touch32 touch64 --rounds 2 -- --steps 3 --warmup 1 --method hh
echo ALL_DONE
