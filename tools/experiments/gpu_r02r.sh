# Round 2, session D: PMC refresh of the default bench (FETCH_SIZE / WRITE_SIZE, separate
# passes, one full cycle) and of the Chebyshev(8) config; the box's counter list.
OUT=gpurun_out/r02r
source tools/gpu_lib.sh
step counters 120 rocprofv3 -L
pmc pmc_fetch FETCH_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag
pmc pmc_write WRITE_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag
pmc pmc_fetch_cheb FETCH_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag --prec cheb
pmc pmc_write_cheb WRITE_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag --prec cheb
echo ALL_DONE
