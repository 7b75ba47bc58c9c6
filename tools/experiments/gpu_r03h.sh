# Round 3, call h: the fused Chebyshev epilogue mismatch at >= 2048^2 -- where
# and whether it is deterministic (ACC_NONE apply twice, ACC_NORM cycle start).
OUT=gpurun_out/r03h
source tools/gpu_lib.sh
step cheb_diag 300 python -u tools/cheb_diag.py --grids 1024 2048 4096 --degrees 8
step cheb_diag2 300 python -u tools/cheb_diag.py --grids 4096 --degrees 2 8
echo ALL_DONE
