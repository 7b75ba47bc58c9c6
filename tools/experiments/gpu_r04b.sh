# Round 4, second call: the multi-rank tests with the corrected launch count
# (the solve's ||b|| is one k_proj launch), the column-cache kernel k_mgs_wpc
# (w+column) in every resident test, A/B against k_mgs_res<12,18> (now with V_q
# default-policy loads) at 2896^2 and 2048^2, its split, rocprof stats, and
# PMC FETCH/WRITE passes at 2896^2 / 2048^2 / 1448^2 (the per-GPU kernels of
# the 2 / 4 / 8-GPU splits).
OUT=gpurun_out/r04b
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
step t_resident 600 $T tests/test_gpu_resident.py
step t_splits 900 $T tests/test_gpu_splits.py
step t_config4 300 $T tests/test_gpu_configs.py -k "config4"
step t_multirank 300 $T -s tests/test_gpu_multirank.py -k "rccl or graphs"
step bench_2896 300 python -u bench.py --grid 2896 --no-cpu --no-configs
step bench_2896_old 300 python -u bench.py --grid 2896 --no-cpu --no-configs --tune 21=0
step bench_2896b 300 python -u bench.py --grid 2896 --no-cpu --no-configs
step bench_2896_oldb 300 python -u bench.py --grid 2896 --no-cpu --no-configs --tune 21=0
step bench_2048 300 python -u bench.py --grid 2048 --no-cpu --no-configs
step bench_2048_old 300 python -u bench.py --grid 2048 --no-cpu --no-configs --tune 21=0
step bench_1448 300 python -u bench.py --grid 1448 --no-cpu --no-configs
step bench_1448_pc 300 python -u bench.py --grid 1448 --no-cpu --no-configs --tune 21=1
step split_2896 300 python -u tools/res_split.py --grid 2896 --method both
step trace_2896 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_2896" -o t2896 --output-format csv -- python3 bench.py --grid 2896 --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_fetch_2896 FETCH_SIZE python3 bench.py --grid 2896 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_2896 WRITE_SIZE python3 bench.py --grid 2896 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_fetch_2048 FETCH_SIZE python3 bench.py --grid 2048 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_2048 WRITE_SIZE python3 bench.py --grid 2048 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_fetch_1448 FETCH_SIZE python3 bench.py --grid 1448 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_1448 WRITE_SIZE python3 bench.py --grid 1448 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
