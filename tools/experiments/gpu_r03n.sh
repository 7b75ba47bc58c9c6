# Round 3, call n: the Chebyshev pass with the pre-loop drain (no vmcnt(0) per
# FAST trip): Chebyshev tests, config-3 bench + rocprof; host wait probe; the
# default bench (spin wait, PCIe-inclusive diagnostic); multi-rank drift per
# residual tier; config 4 against the reference's own 8192^2 cycle.
OUT=gpurun_out/r03n
source tools/gpu_lib.sh
step cheb_tests 500 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "cheb or precond or Cheb or config3 or epilogue or stencil"
step bench_cheb 300 python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs
step rocprof_cheb 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cheb -o prof_cheb --output-format csv -- python -u bench.py --prec cheb --steps 2 --warmup 1 --no-cpu --no-configs --no-diag
step wait_probe 200 python -u tools/host_wait_probe.py
step bench_default 500 python -u bench.py
step multirank_dev 300 python -u tools/multirank_dev.py
step config4 400 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread -k config4
echo ALL_DONE
