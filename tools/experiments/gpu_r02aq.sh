# Round 2, session E: sanity of the final in-tree build (suite, smoke, short default bench).
OUT=gpurun_out/r02aq
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python -u bench.py --no-cpu --steps 5 --warmup 1
echo ALL_DONE
