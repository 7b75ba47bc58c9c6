# Round 2, session E: reflection chains with RW 90 / WB 6 (whole 4096^2 slab on chip) while the
# MGS-R step keeps 88 / 8: full GPU suite, smoke, Householder A/B against 88 / 8 (hh88),
# bench lines, rocprof stats of the Householder bench.
OUT=gpurun_out/r02al
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ab4096hh 600 python -u tools/ab_lib.py --variants base hh88 --rounds 3 -- --steps 3 --warmup 1 --no-diag --method hh
step bench_default 400 python -u bench.py --steps 20 --warmup 5
step bench_hh 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --method hh
step trace_hh 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_hh" -o hh --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag --method hh
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-diag
echo ALL_DONE
