# Round 3, call j: evidence of the tree after the stencil-stage pass: the
# default bench (headline + config legs + reference CPU thread sweep) and a
# rocprof of the headline.
OUT=gpurun_out/r03j
source tools/gpu_lib.sh
step bench_default 500 python -u bench.py
step rocprof_default 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o prof_default --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu --no-configs --no-diag
echo ALL_DONE
