# Round 3, call s: the 1024^2 leg inside the bench (44 ms per cycle) vs alone
# (36.7): after a closed 4096^2 context; and the true-residual warmup again.
OUT=gpurun_out/r03s
source tools/gpu_lib.sh
step l1024_pre 200 python -u tools/leg_order.py --grid 1024 --cycles 3 --pre-grid 4096 --legs identity identity
step l1024_pre_hist 200 python -u tools/leg_order.py --grid 1024 --cycles 3 --pre-grid 4096 --hist-warm --legs identity identity
step l4096_hist 200 python -u tools/leg_order.py --hist-warm --legs cheb cheb
step l4096_pre_hist 200 python -u tools/leg_order.py --pre-grid 4096 --hist-warm --legs cheb cheb
echo ALL_DONE
