# resident launches over the device exchange (2 ranks on one GPU), MGS-R and Householder
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_xgmi.py -x -v --timeout 150 --timeout-method thread > gpurun_out/xgmi_hh_tests.log 2>&1 && echo TESTS_OK
