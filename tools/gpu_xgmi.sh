#!/bin/bash
# Device-exchange back-end on the 1-GPU box: its tests, the full GPU suite, and
# the per-collective cost probe.  Every GPU step bounded, chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_xgmi.py -x -q > gpurun_out/xgmi_tests.log 2>&1 && echo XGMI_TESTS_OK \
&& timeout -k 10 300 python tools/xchg_latency.py > gpurun_out/xchg_lat.json 2> gpurun_out/xchg_lat.err && cat gpurun_out/xchg_lat.json \
&& timeout -k 10 1200 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_all.log 2>&1 && echo GPU_ALL_OK
rc=$?
tail -15 gpurun_out/xgmi_tests.log
tail -5 gpurun_out/gpu_all.log 2>/dev/null
exit $rc
