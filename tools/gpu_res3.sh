# w-only resident variant: parity, then A/B at 4096^2 and 2048^2
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 150 --timeout-method thread > gpurun_out/res3_tests.log 2>&1 && echo RES_TESTS_OK &&
timeout -k 10 500 python -u tools/tune.py --grid 4096 --m 95 --rounds 2 --variants res=1 res=1:wo=1 --out gpurun_out/tune3_4096.json > gpurun_out/tune3_4096.log 2>&1 && echo T4096_OK &&
timeout -k 10 300 python -u tools/tune.py --grid 2048 --m 95 --rounds 2 --variants res=0 res=1 res=1:wo=1 --out gpurun_out/tune3_2048.json > gpurun_out/tune3_2048.log 2>&1 && echo T2048_OK
