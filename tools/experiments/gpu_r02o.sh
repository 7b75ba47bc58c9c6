# Round 2, session D: two-hop grouped all-gather (group leaders) vs the flat sweep.
OUT=gpurun_out/r02o
source tools/gpu_lib.sh
step tests 900 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_solver.py tests/test_gpu_configs.py tests/test_gpu_xgmi.py -v --timeout 200 --timeout-method thread
step ab1024 600 python -u tools/ab_lib.py --variants base flat --rounds 3 -- --steps 10 --warmup 2 --grid 1024 --no-diag
step ab2048 600 python -u tools/ab_lib.py --variants base flat --rounds 2 -- --steps 5 --warmup 1 --grid 2048 --no-diag
step ab4096 600 python -u tools/ab_lib.py --variants base flat --rounds 2 -- --steps 3 --warmup 1 --no-diag
step split 300 python -u tools/res_split.py --grid 1024 --method mgsr
echo ALL_DONE
