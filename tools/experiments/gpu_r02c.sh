# Round 2, session C: Householder UP chain without a reduction in its last pass
# (tail norm after the loop) -- parity suites, in-kernel split, HH and MGS-R bench.
OUT=gpurun_out/r02c
source tools/gpu_lib.sh
step parity 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_configs.py tests/test_gpu_solver.py tests/test_gpu_xgmi.py tests/test_gpu_multirank.py -v --timeout 120 --timeout-method thread
step split4096 300 python -u tools/res_split.py --grid 4096
step bench_hh 300 python -u bench.py --method hh --no-cpu --steps 5 --warmup 1
step bench_mgs 300 python -u bench.py --no-cpu --steps 5 --warmup 1
echo ALL_DONE
