# Round 3, call e: where the buffer-addressed FAST steps of the Chebyshev pass
# differ from the oracle (1024..4096, degrees 1 / 4 / 8), and the per-solve
# overhead of short solves at 1024^2 (the bench's config legs).
OUT=gpurun_out/r03e
source tools/gpu_lib.sh
step cheb_diag 300 python -u tools/cheb_diag.py --grids 256 1024 2048 4096 --degrees 1 4 8
step overhead_1024 200 python -u tools/solve_overhead.py --grid 1024 --prof-every 16
step overhead_1024_noprof 200 python -u tools/solve_overhead.py --grid 1024
echo ALL_DONE
