#!/bin/bash
# round 5: the prefetching small-slab blocked builds (parity + bench), the HH
# reference-order norms, the CG/BiCGSTAB histories.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${TAG:-r05d}
mkdir -p $out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_blocked.py \
  "tests/test_gpu_solver.py::test_short_recurrence_history_vs_reference" \
  "tests/test_gpu_solver.py::test_hh_verr_two_sided_with_reference_order_norms" > $out/tests.txt 2>&1
rc=$?; grep -E "passed|failed|\[blocked|\[hh|\[pcg|\[pbicg" $out/tests.txt | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for g in ${GRIDS:-1024 1448}; do
  for s in ${BLOCKS:-2 4}; do
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
# 4096^2: the Infinity-Cache policy of the blocked w-only build's second dot slot
for v in base q1c0 q1c64 q1c90; do
  if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$PWD/gmres_amd/lib/variants/$v; fi
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --grid 4096 --no-cpu --no-configs \
    --tune 23=2 > $out/bench_4096_s2_$v.json 2> $out/bench_4096_s2_$v.err || exit $?
  python - "$out/bench_4096_s2_$v.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sp = d.get("diagnostics", {}).get("resident_split_per_unit_us", {}).get("mgs_step", {})
print("4096 S 2", sys.argv[2], "it/s", round(d["value"], 1), "frac", d["roofline"].get("frac"), "split", sp)
PY
done
