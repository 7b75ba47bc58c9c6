#!/bin/bash
# round 5, last tree: the whole GPU suite, smoke and the default bench line.
OUT=gpurun_out/${TAG:-r05zz}
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
step gpu_tests 900 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests -m gpu
tail -3 $OUT/gpu_tests.out
step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -3 $OUT/smoke.out
step bench_default 500 python -u bench.py
tail -c 200 $OUT/bench_default.out
echo ALL_DONE
