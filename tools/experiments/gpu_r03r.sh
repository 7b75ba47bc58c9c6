# Round 3, call r: a true-residual warmup makes the following Chebyshev(8)
# cycles slower (398.7 vs 391.9 ms) -- kernel statistics of both, to see
# whether a kernel or the gaps between them grew.
OUT=gpurun_out/r03r
source tools/gpu_lib.sh
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step prof_plain 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_plain -o plain --output-format csv -- python -u tools/leg_order.py --legs cheb
step prof_hist 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_hist -o hist --output-format csv -- python -u tools/leg_order.py --hist-warm --legs cheb
echo ALL_DONE
