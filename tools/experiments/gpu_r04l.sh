# Round 4: same-device rehearsals on the two-wave column cache (2 ranks x 128
# workgroups at 2896^2 = the 2-GPU / config-4 load per workgroup; 4 x 64 at
# 2048^2 = the 4-GPU load), resident steps on, their PMC-backed roofline.
OUT=gpurun_out/r04l
source tools/gpu_lib.sh
B="python -u bench.py --no-cpu --no-configs"
step reh2_2896 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh4_2048 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
echo ALL_DONE
