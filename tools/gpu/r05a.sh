#!/bin/bash
# round 5, first GPU pass of the blocked-projection MGS step: its parity tests,
# a strict-path sanity subset, then S = 1 / 2 / 4 bench points at 1024^2, 1448^2, 4096^2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05a
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_blocked.py tests/test_gpu_runtime.py "tests/test_gpu_solver.py::test_short_recurrence_history_vs_reference" \
  > gpurun_out/r05a/blocked_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/r05a/blocked_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py \
  tests/test_gpu_configs.py -k "not config4" > gpurun_out/r05a/strict_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r05a/strict_tests.txt
[ $rc -eq 0 ] || exit $rc
for g in 1024 1448 4096; do
  for s in 1 2 4; do
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --grid $g --no-cpu --no-configs \
      --tune 23=$s > gpurun_out/r05a/bench_${g}_s${s}.json 2> gpurun_out/r05a/bench_${g}_s${s}.err || exit $?
    python - "$g" "$s" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r05a/bench_{sys.argv[1]}_s{sys.argv[2]}.json").read().strip().splitlines()[-1])
sp = d.get("diagnostics", {}).get("resident_split_per_unit_us", {})
print(sys.argv[1], "S", sys.argv[2], "it/s", d["value"], "frac", d["roofline"]["frac"], "split", json.dumps(sp)[:200])
PY
  done
done
