# resident Householder chains: parity (resident + solver + device-exchange suites), then bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_solver.py tests/test_gpu_xgmi.py -x -v --timeout 150 --timeout-method thread > gpurun_out/hhres_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u bench.py --method hh --no-cpu > gpurun_out/hhres_bench_hh.json 2> gpurun_out/hhres_bench_hh.err && echo BENCH_HH_OK && cat gpurun_out/hhres_bench_hh.json &&
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/hhres_bench_mgs.json 2> gpurun_out/hhres_bench_mgs.err && echo BENCH_MGS_OK && cat gpurun_out/hhres_bench_mgs.json &&
timeout -k 10 200 python -u bench.py --grid 1024 --steps 3 --no-cpu > gpurun_out/hhres_bench_1024.json 2> gpurun_out/hhres_bench_1024.err && echo BENCH_1024_OK && cat gpurun_out/hhres_bench_1024.json
