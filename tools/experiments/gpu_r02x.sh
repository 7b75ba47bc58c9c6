# Round 2, session E: Householder step fusion (GK_TUNE_HH_FUSE): resident + solver
# + full-size config-5 tests, HH bench, rocprof kernel stats of the HH bench.
OUT=gpurun_out/r02x
source tools/gpu_lib.sh
step gpu_tests 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_solver.py tests/test_gpu_configs.py tests/test_gpu_xgmi.py tests/test_gpu_multirank.py -m gpu -v --timeout 200 --timeout-method thread
step bench_hh 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --method hh
step trace_hh 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_hh" -o hh --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag --method hh
echo ALL_DONE
