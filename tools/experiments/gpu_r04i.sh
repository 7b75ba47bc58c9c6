# Round 4: the device-exchange step graphs with in-process ranks (the local
# group's contexts now replay too), then an A/B of k_mgs_wres pass ordering at
# 4096^2: REV (LDS halves walked lo/regs/hi then hi/regs/lo, so a pass's AXPY
# column starts on the lines the previous pass read last) with the touch depth
# 28 (capped at a half, 19) / 8 / 0, against the default, MGS-R and Householder;
# the column-cache kernel's batch depth 12 / 10 vs 8 at 2896^2.
OUT=gpurun_out/r04i
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs --no-diag"
V=gmres_amd/lib/variants
step t_graphs 300 $T tests/test_gpu_multirank.py -k "graphs" -s
step base_a 120 $B
step rev1 120 env GK_LIB_DIR=$V/rev1 $B
step rev1t8 120 env GK_LIB_DIR=$V/rev1t8 $B
step rev1t0 120 env GK_LIB_DIR=$V/rev1t0 $B
step base_b 120 $B
step rev1_b 120 env GK_LIB_DIR=$V/rev1 $B
step hh_base 120 $B --method hh
step hh_rev1 120 env GK_LIB_DIR=$V/rev1 $B --method hh
step pc_base_a 120 $B --grid 2896
step pc_wb12 120 env GK_LIB_DIR=$V/pcwb12 $B --grid 2896
step pc_wb10 120 env GK_LIB_DIR=$V/pcwb10 $B --grid 2896
step pc_base_b 120 $B --grid 2896
step pc_wb12_b 120 env GK_LIB_DIR=$V/pcwb12 $B --grid 2896
echo ALL_DONE
