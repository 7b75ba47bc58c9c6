# Round 2, session E: flat sweep everywhere (8 granule replicas): full GPU suite, smoke,
# small-kernel A/B at 1024^2 / 2048^2, default bench with the reference CPU baseline,
# Householder / Chebyshev(8) / 1024^2 bench lines, rocprofv3 kernel stats of the default bench.
OUT=gpurun_out/r02ab
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ab1024 500 python -u tools/ab_lib.py --variants base s1 s8 rep16 rep4 hop2 --rounds 2 -- --steps 10 --warmup 2 --no-diag --grid 1024
step ab2048 500 python -u tools/ab_lib.py --variants base s1 rep16 rep4 --rounds 2 -- --steps 5 --warmup 1 --no-diag --grid 2048
step bench_default 400 python -u bench.py --steps 20 --warmup 5
step bench_hh 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --method hh
step bench_cheb 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --prec cheb
step bench_1024 300 python -u bench.py --no-cpu --steps 20 --warmup 5 --grid 1024
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag
step trace4096 300 python -u tools/res_trace.py --grid 4096 --steps 16,48,80
step trace1024 300 python -u tools/res_trace.py --grid 1024 --steps 48
echo ALL_DONE
