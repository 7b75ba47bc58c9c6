# Round 3, call b: the rewritten Chebyshev pass (DPP lane shifts, edge windows
# aligned to the grid's W / E boundaries, no per-point selects, skipped
# prologue levels, 2-deep ring, 2 waves per SIMD): its parity tests, config 3
# bench line, rocprof kernel stats of that bench.
OUT=gpurun_out/r03b
source tools/gpu_lib.sh
step cheb_tests 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "cheb or precond or Cheb or config3 or config_3"
step bench_cheb 300 python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs
step rocprof_cheb 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cheb -o prof_cheb --output-format csv -- python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs --no-diag
echo ALL_DONE
