# Round 4: the column-cache kernel in 512-thread workgroups (two waves per SIMD,
# 32 chunks of w per thread, RX register-cached + 19 LDS-cached column chunks)
# against the 256-thread default at 2896^2 (the 2-GPU / config-4 load), forced
# onto the column cache (--tune 21=1); MGS-R and Householder; the resident tests
# on the 512 build.
OUT=gpurun_out/r04j
source tools/gpu_lib.sh
B="python -u bench.py --no-cpu --no-configs --no-diag --grid 2896"
V=gmres_amd/lib/variants
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
step base_a 120 $B
step a512 120 env GK_LIB_DIR=$V/pc512a $B --tune 21=1
step b512 120 env GK_LIB_DIR=$V/pc512b $B --tune 21=1
step base_b 120 $B
step a512_b 120 env GK_LIB_DIR=$V/pc512a $B --tune 21=1
step b512_b 120 env GK_LIB_DIR=$V/pc512b $B --tune 21=1
step hh_base 120 $B --method hh
step hh_a512 120 env GK_LIB_DIR=$V/pc512a $B --tune 21=1 --method hh
step hh_b512 120 env GK_LIB_DIR=$V/pc512b $B --tune 21=1 --method hh
step b2048_base 120 python -u bench.py --no-cpu --no-configs --no-diag --grid 2048
step b2048_a512 120 env GK_LIB_DIR=$V/pc512a python -u bench.py --no-cpu --no-configs --no-diag --grid 2048 --tune 21=1
step t_res_a512 400 env GK_LIB_DIR=$V/pc512a $T tests/test_gpu_resident.py -k "pc or PC"
echo ALL_DONE
