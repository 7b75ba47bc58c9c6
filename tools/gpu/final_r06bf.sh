# r06bf: the round's last tree -- GPU suite, smoke, the default bench line (with the
# reference CPU baseline), rocprofv3 kernel stats of the default line's headline configuration
OUT=gpurun_out/r06bf
. tools/gpu_lib.sh
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o default --output-format csv -- python3 -u bench.py --no-cpu --no-configs --no-sr --steps 3
