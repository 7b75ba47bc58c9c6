#!/bin/bash
# round 5: the split prefetch (waves that do not poll issue it) on the final tree: blocked /
# split / config tests, a 2-rank 1448^2 rehearsal carrying both opt-in legs (blocked, strict
# prefetch), and the default bench line.
OUT=gpurun_out/r05ar
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
step t_blk 900 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_blocked.py tests/test_gpu_splits.py tests/test_gpu_configs.py
tail -1 $OUT/t_blk.out
step reh2_1448 300 env GK_BENCH_SAME_DEVICE=1 python -u bench.py --no-cpu --no-configs --gpus 2 --grid 1448
python - $OUT/reh2_1448.out <<'PY' || true
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g = d["diagnostics"]
print("reh2_1448 strict", round(d["value"], 1), "blocked", (g.get("blocked_leg") or {}).get("it_s"),
      "strict-prefetch", (g.get("strict_prefetch_leg") or {}).get("it_s"), (g.get("strict_prefetch_leg") or {}).get("error"))
PY
step bench_default 500 python -u bench.py --no-cpu
tail -c 200 $OUT/bench_default.out
echo ALL_DONE
