#!/bin/bash
# round 5: the blocked-step GPU tests (blocked, splits, configs) on the 96 KiB prefetch cap,
# then the default bench line.
OUT=gpurun_out/r05af
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
step t_blk 900 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_blocked.py tests/test_gpu_splits.py tests/test_gpu_configs.py
tail -3 $OUT/t_blk.out
step bench_default 500 python -u bench.py
tail -c 300 $OUT/bench_default.out
echo ALL_DONE
