# Round 4: the column-cache kernels' all-gather poll interval at the 4-GPU load
# on the 16-chunk instantiation (s_sleep 16 default vs 4).
OUT=gpurun_out/r04r
source tools/gpu_lib.sh
B="python -u bench.py --no-cpu --no-configs"
V=gmres_amd/lib/variants
step s16_a 120 $B --grid 2048
step s4_a 120 env GK_LIB_DIR=$V/pcsl4 $B --grid 2048
step s16_b 120 $B --grid 2048
step s4_b 120 env GK_LIB_DIR=$V/pcsl4 $B --grid 2048
step hh_s16 120 $B --grid 2048 --method hh
step hh_s4 120 env GK_LIB_DIR=$V/pcsl4 $B --grid 2048 --method hh
echo ALL_DONE
