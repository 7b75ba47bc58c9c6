# Round 4: more samples of the first-dot fold A/B (same-device rehearsals,
# alternating fold on / off), 2 ranks at 2896^2 and 1448^2, 4 ranks at 2048^2.
OUT=gpurun_out/r04u
source tools/gpu_lib.sh
B="python -u bench.py --no-cpu --no-configs"
for k in 1 2 3; do
  step reh2_on_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
  step reh2_off_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896 --tune 22=0
  step reh4_on_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
  step reh4_off_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048 --tune 22=0
  step reh2s_on_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 1448
  step reh2s_off_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 1448 --tune 22=0
done
echo ALL_DONE
