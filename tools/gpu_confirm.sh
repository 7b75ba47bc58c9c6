# re-entry check: full GPU suite, smoke, default bench line (fresh box, prebuilt tree)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/confirm_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/confirm_smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 400 python -u bench.py > gpurun_out/confirm_bench.json 2> gpurun_out/confirm_bench.err && echo BENCH_OK && cat gpurun_out/confirm_bench.json
