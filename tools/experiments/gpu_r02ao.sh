# Round 2, session E: final evidence of the session's tree: full GPU suite, smoke, bench lines
# for every config (default with the reference CPU baseline), rocprofv3 kernel stats of the
# default / Householder / Chebyshev(8) benches, PMC FETCH_SIZE / WRITE_SIZE passes of the
# default cycle, all-gather trace.
OUT=gpurun_out/r02ao
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python -u bench.py --steps 20 --warmup 5
step bench_hh 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --method hh
step bench_cheb 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --prec cheb
step bench_cbpr2 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --prec cbpr2
step bench_1024 300 python -u bench.py --no-cpu --steps 20 --warmup 5 --grid 1024
step bench_2048 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --grid 2048
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag
step trace_hh 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_hh" -o hh --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag --method hh
step trace_cheb 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_cheb" -o cheb --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag --prec cheb
pmc pmc_fetch FETCH_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag
pmc pmc_write WRITE_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag
step restrace 300 python -u tools/res_trace.py --grid 4096 --steps 16,48,80
echo ALL_DONE
