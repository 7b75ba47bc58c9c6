# Round 2, session D: Householder DOWN chains skip the leading-dot pass for unit inputs.
OUT=gpurun_out/r02t
source tools/gpu_lib.sh
step tests 900 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_solver.py tests/test_gpu_configs.py tests/test_gpu_xgmi.py tests/test_gpu_multirank.py -v --timeout 200 --timeout-method thread -k "hh or householder or verr or config5"
step bench_hh 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --method hh
step split 300 python -u tools/res_split.py --grid 4096 --method hh
echo ALL_DONE
