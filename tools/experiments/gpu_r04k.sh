# Round 4: the two-wave column-cache kernel as the default (2896^2 and 2048^2
# select it): the GPU suite on it, its register split / batch A/B at 2896^2,
# PMC FETCH/WRITE passes at 2896^2 and 2048^2 for the byte model, the bench
# points the scaling prediction reads.
OUT=gpurun_out/r04k
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --no-diag --grid 2896"
V=gmres_amd/lib/variants
step gpu_tests 600 $T tests -m gpu
step base_a 120 $B
step rx4wb5 120 env GK_LIB_DIR=$V/rx4wb5 $B
step rx2wb4 120 env GK_LIB_DIR=$V/rx2wb4 $B
step rx4wb3 120 env GK_LIB_DIR=$V/rx4wb3 $B
step rx0wb6 120 env GK_LIB_DIR=$V/rx0wb6 $B
step base_b 120 $B
step hh_base 120 $B --method hh
step hh_rx4wb5 120 env GK_LIB_DIR=$V/rx4wb5 $B --method hh
step point_2896 120 python -u bench.py --no-cpu --no-configs --grid 2896
step point_2048 120 python -u bench.py --no-cpu --no-configs --grid 2048
step point_1448 120 python -u bench.py --no-cpu --no-configs --grid 1448
pmc pmc_fetch_2896 FETCH_SIZE python3 bench.py --grid 2896 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_2896 WRITE_SIZE python3 bench.py --grid 2896 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_fetch_2048 FETCH_SIZE python3 bench.py --grid 2048 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_2048 WRITE_SIZE python3 bench.py --grid 2048 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
step trace_2896 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_2896" -o t2896 --output-format csv -- python3 bench.py --grid 2896 --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
