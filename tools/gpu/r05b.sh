#!/bin/bash
# round 5: the whole GPU suite on the cleaned-up kernels + the blocked step, then
# S = 1 / 2 / 4 bench points at the per-GPU loads of the 1/2/4/8-GPU splits.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${TAG:-r05b}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests \
  > $out/gpu_tests.txt 2>&1
rc=$?; tail -15 $out/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for g in ${GRIDS:-1024 1448 2048 2896 4096}; do
  for s in 1 2 4; do
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --grid $g --no-cpu --no-configs \
      --tune 23=$s > $out/bench_${g}_s${s}.json 2> $out/bench_${g}_s${s}.err || exit $?
    python - "$out" "$g" "$s" <<'PY'
import json, sys
d = json.loads(open(f"{sys.argv[1]}/bench_{sys.argv[2]}_s{sys.argv[3]}.json").read().strip().splitlines()[-1])
sp = d.get("diagnostics", {}).get("resident_split_per_unit_us", {}).get("mgs_step", {})
print(sys.argv[2], "S", sys.argv[3], "it/s", round(d["value"], 1), "frac", d["roofline"].get("frac"),
      "variant", d["roofline"].get("variant"), "split", sp)
PY
  done
done
