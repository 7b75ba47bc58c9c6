# Resident MGS-R step: parity tests, multi-rank device-exchange tests, then A/B timing
set -o pipefail
echo skip-res-tests &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_xgmi.py tests/test_gpu_solver.py -x -v --timeout 150 --timeout-method thread > gpurun_out/res_tests2.log 2>&1 && echo TESTS2_OK &&
timeout -k 10 300 python -u tools/tune.py --grid 1024 --m 95 --rounds 3 --variants res=0 res=1 --out gpurun_out/tune_res_1024.json > gpurun_out/tune_res_1024.log 2>&1 && echo T1024_OK &&
timeout -k 10 400 python -u tools/tune.py --grid 4096 --m 95 --rounds 2 --variants res=0 res=1 res=1:rr2=8 --out gpurun_out/tune_res_4096.json > gpurun_out/tune_res_4096.log 2>&1 && echo T4096_OK
