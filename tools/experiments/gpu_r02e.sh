# Round 2, session D: v_err by value (reference-order diagnostics), and the
# L2 touch-prefetch during the resident all-gather (GK_RES_TOUCH variants).
OUT=gpurun_out/r02e
source tools/gpu_lib.sh
step verr 400 python -u -m pytest tests/test_gpu_solver.py -v --durations=8 --timeout 200 --timeout-method thread
step ab_touch 900 python -u tools/ab_lib.py --variants base touch8 touch16 touch32 --rounds 2 -- --steps 3 --warmup 1
echo ALL_DONE
