# r06bk: the round's last tree (after the Chebyshev fine line tile) -- GPU suite, smoke, the
# default bench line (with the reference CPU baseline), rocprofv3 kernel stats of config 3
OUT=gpurun_out/r06bk
. tools/gpu_lib.sh
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py
step prof_cheb 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o cheb --output-format csv -- python3 -u bench.py --prec cheb --no-cpu --no-sr --no-configs --steps 2
