# Round 4: the MGS step's column cache with 6 register chunks (25 of 32 cached,
# 9.75 B/unknown; the reflection chains keep 4) against the RX_MGS=4 build at
# 2896^2; the resident / split tests on it; PMC and the bench point at 2896^2.
OUT=gpurun_out/r04y
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
V=gmres_amd/lib/variants
step t_res 900 $T tests/test_gpu_resident.py tests/test_gpu_splits.py -k "not 1448 and not 4096"
step rx6_a 120 $B --grid 2896
step rx4_a 120 env GK_LIB_DIR=$V/rxm4 $B --grid 2896
step rx6_b 120 $B --grid 2896
step rx4_b 120 env GK_LIB_DIR=$V/rxm4 $B --grid 2896
step reh2_rx6 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh2_rx4 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/rxm4 $B --gpus 2 --grid 2896
pmc pmc_fetch_2896 FETCH_SIZE python3 bench.py --grid 2896 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_2896 WRITE_SIZE python3 bench.py --grid 2896 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
step trace_2896 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_2896" -o t2896 --output-format csv -- python3 bench.py --grid 2896 --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
