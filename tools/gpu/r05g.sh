#!/bin/bash
# the r04d configuration (8 processes on one GPU, resident steps forced on) with one
# hardware queue per process and every wait bounded (60 s host watchdog, 20 s device deadlines)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r05g
mkdir -p $out
export PYTHONUNBUFFERED=1 GK_BENCH_SAME_DEVICE=1
GPU_MAX_HW_QUEUES=1 timeout -k 10 400 python -u bench.py --gpus 8 --grid 1448 --steps 2 --warmup 1 --no-cpu \
  --no-configs --collective xgmi --tune 24=60000 > $out/reh8_1448_res.json 2> $out/reh8_1448_res.err
rc=$?; grep -E "collective|warmup|timed|Error|error|failed|FAIL" $out/reh8_1448_res.err | head -30; echo "reh8 res rc=$rc"
tail -c 400 $out/reh8_1448_res.json
exit $rc
