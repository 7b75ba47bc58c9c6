# Round 4: the first-dot fold on the Householder UP chain too -- the split,
# device-exchange, multi-rank and config tests; a 2-rank HH rehearsal.
OUT=gpurun_out/r04v
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
step t_multi 900 $T tests/test_gpu_splits.py tests/test_gpu_xgmi.py tests/test_gpu_multirank.py tests/test_gpu_configs.py tests/test_gpu_resident.py
step reh4_hh_fold 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048 --method hh
step reh4_hh_nofold 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048 --method hh --tune 22=0
echo ALL_DONE
