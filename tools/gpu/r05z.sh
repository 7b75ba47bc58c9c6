#!/bin/bash
# Round 5, final tree: the whole GPU suite, smoke, the default bench line (with its config
# legs and the reference CPU baseline) and its rocprofv3 kernel stats, the equal-load
# strict points, the blocked config-2 step's kernel stats, and same-device rehearsals (2 ranks
# at 2896^2, 4 at 2048^2, 8 at 1448^2 -- each N > 1 line with its blocked leg).
OUT=gpurun_out/${TAG:-r05z}
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
step gpu_tests 900 $T tests -m gpu
tail -3 $OUT/gpu_tests.out
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 500 python -u bench.py
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
step trace_blk1024 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_blk1024" -o blk1024 --output-format csv -- python3 bench.py --grid 1024 --tune 23=4 --steps 3 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
for g in 1024 1448 2048 2896; do step point_$g 150 $B --grid $g; done
step reh2 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 2 --grid 2896
step reh4 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 4 --grid 2048
step reh8 300 env GK_BENCH_SAME_DEVICE=1 $B --gpus 8 --grid 1448 --steps 2 --warmup 1 --collective xgmi --tune 24=60000
echo ALL_DONE
