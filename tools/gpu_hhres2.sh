# resident Householder chains after the head-chunk tail norm: parity, then the HH bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_solver.py -x -v --timeout 150 --timeout-method thread -k "householder or hh or resident" > gpurun_out/hhres2_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u bench.py --method hh --no-cpu > gpurun_out/hhres2_bench_hh.json 2> gpurun_out/hhres2_bench_hh.err && echo BENCH_HH_OK && cat gpurun_out/hhres2_bench_hh.json
