# Round 2, session D (container re-created, libraries rebuilt): full GPU suite,
# smoke, default bench line (with the reference CPU baseline), rocprofv3 stats.
OUT=gpurun_out/r02d
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python -u bench.py --steps 20 --warmup 5
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu
echo ALL_DONE
