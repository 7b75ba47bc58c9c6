# Round 4, final tree: the whole GPU suite, smoke, the default bench line and
# its rocprofv3 kernel stats, same-device rehearsals (2 ranks at 2896^2 twice,
# 4 ranks at 2048^2).
OUT=gpurun_out/r04z
source tools/gpu_lib.sh
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
step gpu_tests 600 $T tests -m gpu
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 500 python -u bench.py
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
step reh2_a 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh2_b 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh4 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
echo ALL_DONE
