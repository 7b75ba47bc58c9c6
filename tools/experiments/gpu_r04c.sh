# Round 4, third call: k_mgs_wpc with 16-chunk batches (MGS) / 12 (reflections)
# against its 8-chunk build (GK_LIB_DIR variant) and against k_mgs_res<12,18>
# (--tune 21=0) at 2896^2 and 2048^2; the fixed resident / config-4 tests;
# same-device rehearsals (2 and 4 ranks) for the collective's per-call cost
# (the scaling prediction's lower bound); PMC of the new kernel at 2896^2.
OUT=gpurun_out/r04c
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
step t_resident 600 $T tests/test_gpu_resident.py
step t_config4 300 $T tests/test_gpu_configs.py -k "config4"
step b2896 120 $B --grid 2896
step b2896_wb8 120 env GK_LIB_DIR=gmres_amd/lib/variants/pcwb8 $B --grid 2896
step b2896_old 120 $B --grid 2896 --tune 21=0
step b2896b 120 $B --grid 2896
step b2896_wb8b 120 env GK_LIB_DIR=gmres_amd/lib/variants/pcwb8 $B --grid 2896
step b2048 120 $B --grid 2048
step b2048_wb8 120 env GK_LIB_DIR=gmres_amd/lib/variants/pcwb8 $B --grid 2048
step b2048_old 120 $B --grid 2048 --tune 21=0
step b2048b 120 $B --grid 2048
step b2048_oldb 120 $B --grid 2048 --tune 21=0
step b1448_pc 120 $B --grid 1448 --tune 21=1
step b1448 120 $B --grid 1448
step b4096 300 $B --steps 3
step reh2_2896 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh4_2048 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
step split_2896 120 python -u tools/res_split.py --grid 2896 --method both
step split_2048 120 python -u tools/res_split.py --grid 2048 --method mgsr
step trace_2896 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_2896" -o t2896 --output-format csv -- python3 bench.py --grid 2896 --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
step trace_2048 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_2048" -o t2048 --output-format csv -- python3 bench.py --grid 2048 --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_fetch_2896 FETCH_SIZE python3 bench.py --grid 2896 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_2896 WRITE_SIZE python3 bench.py --grid 2896 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_fetch_2048 FETCH_SIZE python3 bench.py --grid 2048 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_2048 WRITE_SIZE python3 bench.py --grid 2048 --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
