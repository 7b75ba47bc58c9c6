#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r05f
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_solver.py -k "short_recurrence" > $out/short.txt 2>&1
grep -E "PASSED|FAILED|iterations|AssertionError|assert " $out/short.txt | head -40
bash tools/gpu/r05c.sh
