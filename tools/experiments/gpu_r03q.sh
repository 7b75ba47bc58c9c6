# Round 3, call q: the config legs' slowdown -- profiling events and the
# true-residual warmup toggled one at a time on the same legs.
OUT=gpurun_out/r03q
source tools/gpu_lib.sh
step l4096_plain 200 python -u tools/leg_order.py --legs cheb identity
step l4096_prof 200 python -u tools/leg_order.py --prof 16 --legs cheb identity
step l4096_hist 200 python -u tools/leg_order.py --hist-warm --legs cheb identity
step l4096_both 200 python -u tools/leg_order.py --prof 16 --hist-warm --legs cheb identity
step l1024_plain 200 python -u tools/leg_order.py --grid 1024 --cycles 3 --legs identity identity
step l1024_prof 200 python -u tools/leg_order.py --grid 1024 --cycles 3 --prof 16 --legs identity identity
step l1024_hist 200 python -u tools/leg_order.py --grid 1024 --cycles 3 --hist-warm --legs identity identity
step hh_plain 200 python -u tools/leg_order.py --method hh --legs identity
step hh_prof1 200 python -u tools/leg_order.py --method hh --prof 1 --legs identity
echo ALL_DONE
