# Round 3, final evidence of the tree: full GPU suite, smoke, bench lines
# (default with the reference CPU baseline; Householder, Chebyshev(8), 1024^2),
# rocprofv3 kernel stats of the default / Householder / Chebyshev(8) benches,
# PMC FETCH_SIZE / WRITE_SIZE passes of one default cycle.
OUT=gpurun_out/r03u
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 500 python -u bench.py
step bench_hh 300 python -u bench.py --no-cpu --no-configs --method hh
step bench_cheb 300 python -u bench.py --no-cpu --no-configs --prec cheb
step bench_1024 300 python -u bench.py --no-cpu --no-configs --steps 5 --warmup 2 --grid 1024
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
step trace_hh 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_hh" -o hh --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag --method hh
step trace_cheb 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_cheb" -o cheb --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag --prec cheb
pmc pmc_fetch FETCH_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write WRITE_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
