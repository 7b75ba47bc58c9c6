# Round 2, session D: Chebyshev passes with a D-deep input ring -- bit-exactness
# (kernel + full-size config 3 tests) and depth / JT A/B on config 3.
OUT=gpurun_out/r02g
source tools/gpu_lib.sh
step cheb_tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_multirank.py -v --timeout 200 --timeout-method thread -k "cheb or precond or config3"
step ab_cheb 900 python -u tools/ab_lib.py --variants base cfd1 cfd2 cfd3 cfjt128 cfd2jt128 --rounds 2 -- --steps 3 --warmup 1 --prec cheb
echo ALL_DONE
