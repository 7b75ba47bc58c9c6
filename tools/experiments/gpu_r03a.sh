# Round 3, call a: the full GPU suite, now with the multi-rank production
# variants (tests/test_gpu_splits.py: 2 ranks on one GPU at the production chunk
# load, in-process and IPC), config 4 through the device exchange, the straggler
# test and uneven Chebyshev slabs; then the default bench (config legs + CPU
# thread sweep) and the counter list.
OUT=gpurun_out/r03a
source tools/gpu_lib.sh
step gpu_tests 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step bench_default 500 python -u bench.py
step list_avail 60 rocprofv3 --list-avail
echo ALL_DONE
