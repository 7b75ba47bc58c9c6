# Evidence after RES_RW 64 -> 88 (w-only residency 80 % -> 98 % at 4096^2): full GPU suite,
# bench lines, rocprofv3 kernel trace, PMC passes -> gpurun_out/ev5/
set -o pipefail
mkdir -p gpurun_out/ev5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ev5/gpu_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 400 python -u bench.py > gpurun_out/ev5/bench_default.json 2> gpurun_out/ev5/bench_default.err && echo B0 &&
timeout -k 10 300 python -u bench.py --no-cpu --method hh > gpurun_out/ev5/bench_hh.json 2> gpurun_out/ev5/bench_hh.err && echo B1 &&
timeout -k 10 300 python -u bench.py --no-cpu --prec cheb --degree 8 > gpurun_out/ev5/bench_cheb8.json 2> gpurun_out/ev5/bench_cheb8.err && echo B2 &&
timeout -k 10 300 python -u bench.py --no-cpu --prec cbpr2 > gpurun_out/ev5/bench_cbpr2.json 2> gpurun_out/ev5/bench_cbpr2.err && echo B3 &&
timeout -k 10 200 python -u bench.py --no-cpu --grid 1024 --steps 3 > gpurun_out/ev5/bench_1024.json 2> gpurun_out/ev5/bench_1024.err && echo B4 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/ev5/trace -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-prof > gpurun_out/ev5/trace_bench.json 2> gpurun_out/ev5/trace_bench.err && echo P1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/ev5/pmc_fetch -o fetch --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/ev5/pmc_fetch.log 2>&1 && echo P2 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ev5/pmc_write -o write --output-format csv -- python3 tools/pmc_probe.py > gpurun_out/ev5/pmc_write.log 2>&1 && echo P3
