# Round 4: on N ranks workgroup 0 (the rank-total pusher) polls its granules
# without the s_sleep -- same-device rehearsals, 2 ranks at 2896^2 and 4 at
# 2048^2, against the GK_RES_PUSHER_FAST=0 build.
OUT=gpurun_out/r04s
source tools/gpu_lib.sh
B="python -u bench.py --no-cpu --no-configs"
V=gmres_amd/lib/variants
step reh2_fast_a 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh2_slow_a 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/pf0 $B --gpus 2 --grid 2896
step reh4_fast_a 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
step reh4_slow_a 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/pf0 $B --gpus 4 --grid 2048
step reh2_fast_b 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh2_slow_b 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/pf0 $B --gpus 2 --grid 2896
step reh4_fast_b 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
step reh4_slow_b 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/pf0 $B --gpus 4 --grid 2048
echo ALL_DONE
