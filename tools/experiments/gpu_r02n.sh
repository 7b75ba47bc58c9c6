# Round 2, session D: DPP wave sums on the resident steps' critical path -- parity suites, A/B.
OUT=gpurun_out/r02n
source tools/gpu_lib.sh
step tests 900 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_solver.py tests/test_gpu_configs.py tests/test_gpu_xgmi.py -v --timeout 200 --timeout-method thread
step ab1024 900 python -u tools/ab_lib.py --variants base nodpp --rounds 3 -- --steps 10 --warmup 2 --grid 1024 --no-diag
step ab4096 900 python -u tools/ab_lib.py --variants base nodpp --rounds 2 -- --steps 3 --warmup 1 --no-diag
echo ALL_DONE
