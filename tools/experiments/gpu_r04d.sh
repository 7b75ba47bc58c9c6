# Round 4, fourth call: k_mgs_wpc software-pipelined (batch b+1 in flight while
# b is consumed), 8-chunk batches, against a 4-chunk build and k_mgs_res
# (--tune 21=0) at 2896^2 / 2048^2 / 1448^2; the resident tests; the same-device
# rehearsals now on the resident kernels (2 ranks at 2896^2, 4 at 2048^2, 8 at
# 1448^2: the production per-workgroup loads).
OUT=gpurun_out/r04d
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
step t_resident 600 $T tests/test_gpu_resident.py
step b2896 120 $B --grid 2896
step b2896_wb4 120 env GK_LIB_DIR=gmres_amd/lib/variants/pcwb4 $B --grid 2896
step b2896_old 120 $B --grid 2896 --tune 21=0
step b2896b 120 $B --grid 2896
step b2048 120 $B --grid 2048
step b2048_wb4 120 env GK_LIB_DIR=gmres_amd/lib/variants/pcwb4 $B --grid 2048
step b2048_old 120 $B --grid 2048 --tune 21=0
step b2048b 120 $B --grid 2048
step b1448_pc 120 $B --grid 1448 --tune 21=1
step b1448 120 $B --grid 1448
step b2896_hh 120 $B --grid 2896 --method hh
step b2896_hh_old 120 $B --grid 2896 --method hh --tune 21=0
step split_2896 120 python -u tools/res_split.py --grid 2896 --method both
step reh2_2896 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh4_2048 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
step reh8_1448 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 8 --grid 1448
echo ALL_DONE
