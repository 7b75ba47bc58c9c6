# Round 4: evidence of the tree as it stands -- the default bench line (with
# the reference CPU baseline and the config legs), the Householder and
# Chebyshev(8) lines, the per-GPU loads of the 2/4/8-GPU splits, rocprofv3
# kernel stats of the default and 2896^2 runs; the whole GPU suite first.
OUT=gpurun_out/r04g
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
step gpu_tests 600 $T tests -m gpu
step bench_default 500 python -u bench.py
step bench_hh 300 python -u bench.py --no-cpu --no-configs --method hh
step bench_cheb 300 python -u bench.py --no-cpu --no-configs --prec cheb
step bench_1024 300 python -u bench.py --no-cpu --no-configs --steps 5 --warmup 2 --grid 1024
step bench_2896 120 python -u bench.py --no-cpu --no-configs --grid 2896
step bench_2048 120 python -u bench.py --no-cpu --no-configs --grid 2048
step bench_1448 120 python -u bench.py --no-cpu --no-configs --grid 1448
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
step trace_2896 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_2896" -o t2896 --output-format csv -- python3 bench.py --grid 2896 --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
