# Round 2, session D: resident chunks spread evenly over the workgroups --
# resident/solver/config/multirank suites, skew at 2048^2 / 1024^2 / 4096^2, benches.
OUT=gpurun_out/r02l
source tools/gpu_lib.sh
step tests 900 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_solver.py tests/test_gpu_configs.py tests/test_gpu_multirank.py tests/test_gpu_xgmi.py -v --timeout 200 --timeout-method thread
step skew 300 python -u tools/res_split.py --grid 2048 --method mgsr
step skew1024 300 python -u tools/res_split.py --grid 1024 --method mgsr
step skew4096 300 python -u tools/res_split.py --grid 4096
step bench_2048 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --grid 2048
step bench_1024 300 python -u bench.py --no-cpu --steps 20 --warmup 5 --grid 1024
step bench_default 300 python -u bench.py --no-cpu --steps 10 --warmup 2
echo ALL_DONE
