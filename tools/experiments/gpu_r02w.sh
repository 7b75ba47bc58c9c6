# Round 2, session E: re-verification of the rebuilt tree (container re-created):
# full GPU suite, smoke, default bench with the reference CPU baseline.
OUT=gpurun_out/r02w
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python -u bench.py --steps 20 --warmup 5
echo ALL_DONE
