# Round 4: PMC FETCH/WRITE passes and the bench point at 2048^2 on the 16-chunk
# column-cache kernel (the 4-GPU per-GPU load), for the byte model and the
# scaling prediction.
OUT=gpurun_out/r04q
source tools/gpu_lib.sh
step point_2048 120 python -u bench.py --no-cpu --no-configs --grid 2048
pmc pmc_fetch_2048 FETCH_SIZE python3 bench.py --grid 2048 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_2048 WRITE_SIZE python3 bench.py --grid 2048 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
step trace_2048 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_2048" -o t2048 --output-format csv -- python3 bench.py --grid 2048 --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
