# Round 4: 2-rank same-device rehearsal at 2896^2, the MGS column cache with 6
# (default) vs 4 register chunks, alternating, three samples each.
OUT=gpurun_out/r04za
source tools/gpu_lib.sh
B="python -u bench.py --no-cpu --no-configs"
V=gmres_amd/lib/variants
for k in 1 2 3; do
  step rx6_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
  step rx4_$k 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/rxm4 $B --gpus 2 --grid 2896
done
echo ALL_DONE
