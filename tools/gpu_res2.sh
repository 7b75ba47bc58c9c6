# Resident step v2 (control wave, LDS-resident w, small-grid sizing): parity, multi-rank, A/B timing
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_xgmi.py -x -v --timeout 150 --timeout-method thread > gpurun_out/res2_tests.log 2>&1 && echo RES_TESTS_OK &&
timeout -k 10 200 python -u tools/tune.py --grid 128 --m 95 --rounds 3 --variants res=0 res=1 --out gpurun_out/tune2_128.json > gpurun_out/tune2_128.log 2>&1 && echo T128_OK &&
timeout -k 10 300 python -u tools/tune.py --grid 1024 --m 95 --rounds 3 --variants res=0 res=1 --out gpurun_out/tune2_1024.json > gpurun_out/tune2_1024.log 2>&1 && echo T1024_OK &&
timeout -k 10 400 python -u tools/tune.py --grid 4096 --m 95 --rounds 2 --variants res=1 res=1:lds=0 res=1:rr2=8 --out gpurun_out/tune2_4096.json > gpurun_out/tune2_4096.log 2>&1 && echo T4096_OK &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/res2_all.log 2>&1 && echo ALL_OK
