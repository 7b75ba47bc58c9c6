# Round 2, session D: Chebyshev(8) as ONE temporal-blocked pass (L = 8, occupancy-aware JT):
# bit-exactness suites, config-3 bench, kernel stats.
OUT=gpurun_out/r02i
source tools/gpu_lib.sh
step cheb_tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_multirank.py tests/test_gpu_xgmi.py -v --timeout 200 --timeout-method thread -k "cheb or precond or config3"
step bench_cheb 300 python -u bench.py --no-cpu --steps 5 --warmup 1 --prec cheb
step prof_cheb 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o cheb --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --prec cheb
echo ALL_DONE
