# Round 4: the tree as committed -- the whole GPU suite, smoke, the default
# bench line (reference CPU baseline + config legs) and its rocprofv3 kernel
# stats.
OUT=gpurun_out/r04n
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
step gpu_tests 600 $T tests -m gpu
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 500 python -u bench.py
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
