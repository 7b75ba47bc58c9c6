# Round 2, session A: full GPU suite (incl. the full-size config tests), the
# default bench line with the reference CPU baseline, rocprofv3 kernel trace +
# stats of the bench, PMC FETCH_SIZE / WRITE_SIZE over one full cycle.
OUT=gpurun_out/r02a
source tools/gpu_lib.sh
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
step mall 120 ./tools/mall_probe 4096
step mall2k 120 ./tools/mall_probe 2896
step bench_default 400 python -u bench.py --steps 20 --warmup 5
step trace 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu
pmc pmc_fetch FETCH_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof
pmc pmc_write WRITE_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-prof
echo ALL_DONE
