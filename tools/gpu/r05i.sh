#!/bin/bash
# round 5: the whole GPU suite, smoke, the default bench line and its rocprofv3
# kernel stats on the committed tree; then the paced-touch depth of the 4096^2
# w-only step: 28 (main build) vs 20 / 16 (variants),
# alternating bench lines and FETCH_SIZE / WRITE_SIZE passes over one full cycle.
OUT=gpurun_out/r05i
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
V=$PWD/gmres_amd/lib/variants
step gpu_tests 900 $T tests -m gpu
tail -3 $OUT/gpu_tests.out
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_default 500 python -u bench.py
tail -c 600 $OUT/bench_default.out
step trace_default 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_default" -o default --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-configs --no-prof --no-diag
for k in 1 2; do
  for v in base t20 t16; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    step touch_${v}_$k 150 $B
  done
done
for v in base t20 t16; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
  pmc pmc_fetch_$v FETCH_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
  pmc pmc_write_$v WRITE_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
done
echo ALL_DONE
