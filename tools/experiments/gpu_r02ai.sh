# Round 2, session E: L2 touch-prefetch in the two-array small-slab kernel (GK_RES_TOUCH_SMALL
# 12 / 6 / 0 register chunks): full GPU suite, A/B at 2048^2 (the N=4 slab of 4096^2),
# 2896^2 (~ the N=2 slab) and 1448^2 (~ the N=8 slab).
OUT=gpurun_out/r02ai
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step ab2048 500 python -u tools/ab_lib.py --variants base ts0 ts6 --rounds 3 -- --steps 5 --warmup 1 --no-diag --grid 2048
step ab2896 500 python -u tools/ab_lib.py --variants base ts0 ts6 --rounds 2 -- --steps 3 --warmup 1 --no-diag --grid 2896
step ab1448 500 python -u tools/ab_lib.py --variants base ts0 --rounds 2 -- --steps 5 --warmup 1 --no-diag --grid 1448
echo ALL_DONE
