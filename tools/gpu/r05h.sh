#!/bin/bash
# blocked step: reversed second sweep + default-policy dot loads (main build) against the
# round's first order (blk_fwd variant: forward sweeps, cached dot columns non-temporal)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r05h
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_blocked.py \
  > $out/tests.txt 2>&1
rc=$?; tail -2 $out/tests.txt
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in base blk_fwd; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  for g in 1024 1448 2048 2896; do
    for s in 2 4; do
      timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --grid $g --no-cpu --no-configs \
        --tune 23=$s > $out/b_${g}_s${s}_$v.json 2> $out/b_${g}_s${s}_$v.err || exit $?
      python - "$out/b_${g}_s${s}_$v.json" "$g $s $v $rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sp = d.get("diagnostics", {}).get("resident_split_per_unit_us", {}).get("mgs_step", {})
print(sys.argv[2], "it/s", round(d["value"], 1), "split", sp, flush=True)
PY
    done
  done
done
done
