# Round 2, session D: Chebyshev pass with its levels split over two waves (k_cheb_split,
# variant build GK_CF_SPLIT=1): bit-exactness suites on that build, kernel time, bench.
OUT=gpurun_out/r02v
source tools/gpu_lib.sh
export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/split
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_multirank.py tests/test_gpu_xgmi.py -v --timeout 200 --timeout-method thread -k "cheb or precond or config3"
step prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o split --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag --prec cheb
unset GK_LIB_DIR
step ab 600 python -u tools/ab_lib.py --variants base split --rounds 2 -- --steps 3 --warmup 1 --no-diag --prec cheb
echo ALL_DONE
