#!/bin/bash
# round 5: GPU suite on the four-pusher default build + the capture-failure test, default bench.
OUT=gpurun_out/r05k
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
step gpu_tests 900 $T tests -m gpu
tail -3 $OUT/gpu_tests.out
grep -E "FAIL|capture_failure" $OUT/gpu_tests.out | head
step bench_default 500 python -u bench.py
tail -c 300 $OUT/bench_default.out
echo ALL_DONE
