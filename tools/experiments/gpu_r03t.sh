# Round 3, call t: the timed solve keeps x in HBM (no 134 MB download inside
# the timed region) -- its test, the leg with and without the download, the
# default bench; plus call s's legs (1024^2 after a closed 4096^2 context,
# the true-residual warmup again).
OUT=gpurun_out/r03t
source tools/gpu_lib.sh
step test_keep_x 300 python -u -m pytest tests/test_gpu_solver.py -k "kept_in_hbm or true_residual" -v --timeout 120 --timeout-method thread
step l4096_x 200 python -u tools/leg_order.py --legs identity identity
step l4096_keepx 200 python -u tools/leg_order.py --keep-x --legs identity identity
step l1024_pre 200 python -u tools/leg_order.py --grid 1024 --cycles 3 --pre-grid 4096 --keep-x --legs identity identity
step l4096_hist 200 python -u tools/leg_order.py --hist-warm --keep-x --legs cheb cheb
step bench_default 500 python -u bench.py
echo ALL_DONE
