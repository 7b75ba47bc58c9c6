# Round 4: the 16-chunk column-cache instantiation k_mgs_wpc<16,16,0> (w and its
# whole column in registers, no LDS) for slabs of <= 16 chunks per thread
# (2048^2 = the 4-GPU load) against the 32-chunk kernel (GK_RES_PC_SMALL=0
# build); at 1448^2 forced against k_mgs_res<12,0>; the resident, split and
# multi-rank tests on it.
OUT=gpurun_out/r04p
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
V=gmres_amd/lib/variants
step t_res 600 $T tests/test_gpu_resident.py tests/test_gpu_splits.py tests/test_gpu_configs.py
step s_2048_a 120 $B --grid 2048
step b_2048_a 120 env GK_LIB_DIR=$V/pcs0 $B --grid 2048
step s_2048_b 120 $B --grid 2048
step b_2048_b 120 env GK_LIB_DIR=$V/pcs0 $B --grid 2048
step hh_s_2048 120 $B --grid 2048 --method hh
step hh_b_2048 120 env GK_LIB_DIR=$V/pcs0 $B --grid 2048 --method hh
step pairs_1448 120 $B --grid 1448
step s_1448 120 $B --grid 1448 --tune 21=1
step reh4_2048 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
echo ALL_DONE
