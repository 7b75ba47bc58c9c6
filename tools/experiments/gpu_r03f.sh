# Round 3, call f: the fused Chebyshev epilogues (ACC_NORM at the cycle start,
# ACC_DOT in the Arnoldi step) at 1024..4096 against the per-sweep kernels;
# config-3 bench lines at 1024 and 2048.
OUT=gpurun_out/r03f
source tools/gpu_lib.sh
step epi_tests 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v --timeout 200 --timeout-method thread -k "epilogue"
step bench_cheb_1024 200 python -u bench.py --grid 1024 --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs --no-diag
step bench_cheb_2048 200 python -u bench.py --grid 2048 --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs --no-diag
echo ALL_DONE
