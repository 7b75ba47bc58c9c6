#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r05e
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u tools/gpu/diag_pcg.py > $out/diag_pcg.txt 2>&1; cat $out/diag_pcg.txt
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_blocked.py \
  > $out/tests.txt 2>&1
rc=$?; tail -3 $out/tests.txt
[ $rc -eq 0 ] || exit $rc
for g in 1024 1448; do
  for s in 2 4; do
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --grid $g --no-cpu --no-configs \
      --tune 23=$s > $out/bench_${g}_s${s}.json 2> $out/bench_${g}_s${s}.err || exit $?
    python - "$out" "$g" "$s" <<'PY'
import json, sys
d = json.loads(open(f"{sys.argv[1]}/bench_{sys.argv[2]}_s{sys.argv[3]}.json").read().strip().splitlines()[-1])
sp = d.get("diagnostics", {}).get("resident_split_per_unit_us", {}).get("mgs_step", {})
print(sys.argv[2], "S", sys.argv[3], "it/s", round(d["value"], 1), "frac", d["roofline"].get("frac"), "split", sp)
PY
  done
done
