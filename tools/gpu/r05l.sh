#!/bin/bash
# round 5: the 4096^2 w-only MGS step holding the whole slab (89 + 39 chunks, main build)
# against rounds 1-4's 88 + 38 (variant rw88: 2 chunks per workgroup streamed), alternating,
# three samples each; then the resident / config tests and the blocked 4096^2 points (S = 2, 4)
# on the reversed-second-sweep build.
OUT=gpurun_out/r05l
cd "$GRAFT_REPO_ROOT" || exit 1
source tools/gpu_lib.sh
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider"
B="python -u bench.py --no-cpu --no-configs"
V=$PWD/gmres_amd/lib/variants
step t_res 600 $T tests/test_gpu_resident.py tests/test_gpu_configs.py tests/test_gpu_splits.py
tail -2 $OUT/t_res.out
for k in 1 2 3; do
  for v in base rw88; do
    if [ $v = base ]; then unset GK_LIB_DIR; else export GK_LIB_DIR=$V/$v; fi
    step ab_${v}_$k 150 $B
    python - $OUT/ab_${v}_$k.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 2), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"], d["check"]["pass"])
PY
  done
done
unset GK_LIB_DIR
for s in 2 4; do
  step blk4096_s$s 200 $B --tune 23=$s
  python - $OUT/blk4096_s$s.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d["value"], 2), d["roofline"]["per_projection_us"],
      d["diagnostics"]["resident_split_per_unit_us"]["mgs_step"], d["check"]["pass"])
PY
done
pmc pmc_fetch_base FETCH_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
pmc pmc_write_base WRITE_SIZE python3 bench.py --steps 1 --warmup 0 --no-cpu --no-configs --no-prof --no-diag
echo ALL_DONE
