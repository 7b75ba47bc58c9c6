# Round 2, session E: touch depth MGS-R 28 / Householder 24 as defaults: full GPU suite,
# smoke, A/B against the old 32/32 and Householder 16 / 20, bench lines for every config
# (default with the reference CPU baseline), rocprofv3 kernel stats, PMC passes of the
# default bench, all-gather trace.
OUT=gpurun_out/r02ah
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ab4096 600 python -u tools/ab_lib.py --variants base old3232 --rounds 3 -- --steps 3 --warmup 1 --no-diag
step ab4096hh 600 python -u tools/ab_lib.py --variants base old3232 hh16 hh20 --rounds 2 -- --steps 3 --warmup 1 --no-diag --method hh
step bench_default 400 python -u bench.py --steps 20 --warmup 5
step bench_hh 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --method hh
step bench_cheb 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --prec cheb
step bench_cbpr2 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --prec cbpr2
step bench_1024 300 python -u bench.py --no-cpu --steps 20 --warmup 5 --grid 1024
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag
step trace_hh 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_hh" -o hh --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag --method hh
pmc pmc_fetch FETCH_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag
pmc pmc_write WRITE_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof --no-diag
step restrace 300 python -u tools/res_trace.py --grid 4096 --steps 16,48,80
step restrace_rot0 300 env GK_LIB_DIR=gmres_amd/lib/variants/rot0 python -u tools/res_trace.py --grid 4096 --steps 32,64
step restrace_rot1 300 env GK_LIB_DIR=gmres_amd/lib/variants/rot1 python -u tools/res_trace.py --grid 4096 --steps 32,64
echo ALL_DONE
