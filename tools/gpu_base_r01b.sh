# Re-entry baseline: GPU tests + default bench + 1024 bench (each step time-limited, stop at first failure)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/base_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 400 python bench.py > gpurun_out/base_bench4096.json 2> gpurun_out/base_bench4096.err && echo B4096_OK &&
timeout -k 10 200 python bench.py --grid 1024 --steps 3 --no-cpu > gpurun_out/base_bench1024.json 2> gpurun_out/base_bench1024.err && echo B1024_OK
