# Round 4: on N ranks only workgroup 0 (the rank-total pusher) sweeps the local
# granules; the others wait on the rank totals alone.  Multi-rank tests, then
# same-device rehearsals against the GK_RES_SWEEP_ALL=1 build (alternating).
OUT=gpurun_out/r04x
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
V=gmres_amd/lib/variants
step t_multi 900 $T tests/test_gpu_splits.py tests/test_gpu_xgmi.py tests/test_gpu_multirank.py tests/test_gpu_configs.py
for k in 1 2; do
  step reh2_one_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
  step reh2_all_$k 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/sweepall $B --gpus 2 --grid 2896
  step reh4_one_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
  step reh4_all_$k 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/sweepall $B --gpus 4 --grid 2048
  step reh2s_one_$k 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 1448
  step reh2s_all_$k 300 env GK_BENCH_SAME_DEVICE=1 GK_LIB_DIR=$V/sweepall $B --gpus 2 --grid 1448
done
echo ALL_DONE
