# Round 4: the first dot's rank totals inside the MGS step launch on N ranks
# (GK_TUNE_RES_FOLD, one k_xchg launch fewer per Arnoldi step) -- the split,
# device-exchange, multi-rank and config tests on it, then same-device
# rehearsals fold on / off.
OUT=gpurun_out/r04t
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
step t_multi 900 $T tests/test_gpu_splits.py tests/test_gpu_xgmi.py tests/test_gpu_multirank.py tests/test_gpu_configs.py
step reh2_fold 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh2_nofold 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896 --tune 22=0
step reh4_fold 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
step reh4_nofold 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048 --tune 22=0
step reh2_fold_b 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh4_fold_b 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
echo ALL_DONE
