# Round 4: the two-wave column-cache kernel's all-gather poll interval
# (s_sleep units between unanswered polls: 16 default, 8, 4) at 2896^2 and
# 2048^2, MGS-R and Householder.
OUT=gpurun_out/r04m
source tools/gpu_lib.sh
B="python -u bench.py --no-cpu --no-configs"
V=gmres_amd/lib/variants
for g in 2896 2048; do
  step s16_${g}_a 120 $B --grid $g
  step s8_${g} 120 env GK_LIB_DIR=$V/pcsl8 $B --grid $g
  step s4_${g} 120 env GK_LIB_DIR=$V/pcsl4 $B --grid $g
  step s16_${g}_b 120 $B --grid $g
  step s4_${g}_b 120 env GK_LIB_DIR=$V/pcsl4 $B --grid $g
done
step hh_s16 120 $B --grid 2896 --method hh
step hh_s4 120 env GK_LIB_DIR=$V/pcsl4 $B --grid 2896 --method hh
step reh2_s16 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh2_s4 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/pcsl4 $B --gpus 2 --grid 2896
echo ALL_DONE
