# Round 3, closing check of the tree: the full GPU suite (with the driver's
# two-rank bench line as a test), smoke, the default bench line.
OUT=gpurun_out/r03z
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 500 python -u bench.py
echo ALL_DONE
