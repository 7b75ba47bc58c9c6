# Round 4: graph replay of the device exchange's launch path -- the new
# bit-identity test, then same-device rehearsals with the resident step off
# (GK_TUNE_RES=0), step graphs on and off (2 ranks at 2896^2, 4 at 2048^2).
OUT=gpurun_out/r04h
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
step t_graphs 300 $T tests/test_gpu_multirank.py -k "graphs" -s
step reh2_launch_graph 200 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896 --tune 8=0
step reh2_launch_nograph 200 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896 --tune 8=0 --tune 19=0
step reh4_launch_graph 200 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048 --tune 8=0
step reh4_launch_nograph 200 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048 --tune 8=0 --tune 19=0
echo ALL_DONE
